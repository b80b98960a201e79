// handshake_kernels.hip -- batched Noise handshakes on gfx950 (SURVEY.md
// §8(f) rank 4: "batched X25519 / BLAKE2b on the GPU for mass handshakes").
//
// N sessions that run the same handshake pattern in the same role advance in
// lockstep: one lane per session, one kernel per token of the message
// (handshake_batch.hip drives the token program).  Every per-session value
// stays in HBM between kernels in an HsSession row (384 B, AoS: a lane loads
// its own row with dwordx4 loads; the work per token -- an X25519 ladder or
// a dozen BLAKE2b compressions -- dwarfs the 384 B).  The values that are the
// same for every session of a batch -- the token program, HasKey(), the
// handshake-phase nonce n, message cursors -- live on the host and arrive as
// kernel arguments, so the kernels carry no per-session control state beyond
// a sticky status word: a session whose message failed (bad tag, bad length)
// is skipped by every later kernel and keeps its failure code.
//
// Semantics follow the spec-correct host HandshakeState (host/handshake.cpp,
// pinned by the reference's tests/vectors), i.e. Noise rev34 §5.2-5.3 with
// the reference's surface (noise.cpp:441-1100): MixKey / MixHash /
// MixKeyAndHash / EncryptAndHash / DecryptAndHash / Split over BLAKE2b,
// X25519 and ChaChaPoly with AD = h.
#include "blake2b_device.hpp"
#include "launchers.hpp"
#include "x25519_device.hpp"

namespace noise_amd {

namespace {

__device__ __forceinline__ void load_words(uint32_t *w, const HsSession *row, int word0, int n) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint32_t *>(row) + word0);
  for (int q = 0; q < n / 4; ++q) {
    const u32x4 v = p[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}
__device__ __forceinline__ void store_words(HsSession *row, int word0, const uint32_t *w, int n) {
  u32x4 *p = reinterpret_cast<u32x4 *>(reinterpret_cast<uint32_t *>(row) + word0);
  for (int q = 0; q < n / 4; ++q) p[q] = u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
}

constexpr int kWordCk = 0, kWordH = 16, kWordK = 32, kWordStatus = 40, kWordKeys = 48;
static_assert(sizeof(HsSession) == 384, "HsSession layout");

__device__ __forceinline__ void load_key(uint32_t w[8], const HsSession *row, int which) {
  load_words(w, row, kWordKeys + 8 * which, 8);
}
__device__ __forceinline__ void store_key(HsSession *row, int which, const uint32_t w[8]) {
  store_words(row, kWordKeys + 8 * which, w, 8);
}

__device__ __forceinline__ uint8_t *span_ptr(const HsSpan &s, uint64_t i) {
  return s.base + (s.off ? s.off[i] : i * s.stride) + s.add;
}
__device__ __forceinline__ int64_t span_len(const HsSpan &s, uint64_t i) {
  return s.len ? (int64_t)s.len[i] + s.len_adj : (int64_t)s.len_u;
}

__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, int64_t n) {
  for (int64_t b = 0; b < n; ++b) dst[b] = src[b];
}
__device__ __forceinline__ void words_to_bytes(uint8_t *dst, const uint32_t *w, int nbytes) {
  for (int b = 0; b < nbytes; ++b) dst[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}
__device__ __forceinline__ void bytes_to_words(uint32_t *w, const uint8_t *src, int nbytes) {
  for (int j = 0; j < nbytes / 4; ++j) w[j] = ld_bytes(src + 4 * j, 4);
}

// MixKey(ikm): (ck, temp_k) = HKDF(ck, ikm, 2); k = temp_k[0..32)
// (noise.cpp:463-472; the host resets n to 0)
__device__ __forceinline__ void mix_key(HsSession *row, const uint32_t ikm[8], int ilen) {
  uint32_t ck[16], o1[16], o2[16], o3[16];
  load_words(ck, row, kWordCk, 16);
  b2::hkdf(ck, ikm, ilen, 2, o1, o2, o3);
  store_words(row, kWordCk, o1, 16);
  store_words(row, kWordK, o2, 8);
}

__device__ __forceinline__ bool live(const HsSession *row) {
  return reinterpret_cast<const uint32_t *>(row)[kWordStatus] == 0u;
}
__device__ __forceinline__ void fail(HsSession *row, uint32_t code) {
  reinterpret_cast<uint32_t *>(row)[kWordStatus] = code;
}

#define NOISE_HS_ROW()                                    \
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x; \
  if (i >= n) return;                                     \
  HsSession *row = S + i;                                 \
  if (!live(row)) return;

}  // namespace

// InitializeSymmetric (h = ck = h0, the protocol-name hash, host-computed
// since it is the same for every session) + MixHash(prologue_i).
__global__ __launch_bounds__(64) void k_hs_init(HsSession *S, uint64_t n, HsWords16 h0,
                                                HsSpan prologue) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  HsSession *row = S + i;
  uint32_t h[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) h[j] = h0.w[j];
  store_words(row, kWordCk, h, 16);
  const int64_t len = prologue.base ? span_len(prologue, i) : 0;
  b2::mix_hash_mem(h, prologue.base ? span_ptr(prologue, i) : nullptr, len);
  store_words(row, kWordH, h, 16);
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  store_words(row, kWordStatus, z, 8);
}

// Install key `which` for every session: from src (n x 32 bytes at src_stride),
// or -- src == NULL -- a fresh ephemeral from the device DRBG: the first 32
// bytes of ChaCha20(seed, counter = drbg_ctr, nonce = i), seed 32 bytes from
// the OS (getrandom) per call, so every session's key is an independent
// ChaCha20 output block under a fresh key.  derive_pk: key[which + 1] = X25519(key, 9).
__global__ __launch_bounds__(64) void k_hs_set_key(HsSession *S, uint64_t n, int which,
                                                   const uint8_t *src, uint64_t src_stride,
                                                   HsWords8 seed, uint32_t drbg_ctr,
                                                   int derive_pk) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  HsSession *row = S + i;
  uint32_t k[8];
  if (src) {
    bytes_to_words(k, src + i * src_stride, 32);
  } else {
    uint32_t blk[16];
    chacha20_block(seed.w, drbg_ctr, (uint32_t)i, (uint32_t)(i >> 32), blk);
#pragma unroll
    for (int j = 0; j < 8; ++j) k[j] = blk[j];
  }
  store_key(row, which, k);
  if (derive_pk) {  // fixed-base public key (edwards25519 table, x25519_device.hpp)
    uint32_t pk[8];
    x25519::base_scalarmult(pk, k);
    store_key(row, which + 1, pk);
  }
}

// Copy key slots [which, which + count) of row 0 to every row (a key shared by
// all sessions -- a server's static key -- is derived once, by row 0).
__global__ __launch_bounds__(64) void k_hs_bcast_key(HsSession *S, uint64_t n, int which,
                                                     int count) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i == 0 || i >= n) return;
  for (int c = 0; c < count; ++c) {
    uint32_t k[8];
    load_key(k, S, which + c);
    store_key(S + i, which + c, k);
  }
}

// The "e" token and the pre-message keys: optionally move key `which`
// between the session row and the message (io: 0 none, 1 write into msg,
// 2 read from msg; a read also needs msg_len >= cursor + 32, checked by
// k_hs_check_len), then MixHash(key) and, in psk mode, MixKey(key).  A
// fresh ephemeral for a write is installed first by k_hs_set_key.
__global__ __launch_bounds__(64) void k_hs_key_token(HsSession *S, uint64_t n, int which, int io,
                                                     HsSpan msg, int hash, int key) {
  NOISE_HS_ROW();
  uint32_t kv[8];
  if (io == 2) {
    bytes_to_words(kv, span_ptr(msg, i), 32);
    store_key(row, which, kv);
  } else {
    load_key(kv, row, which);
    if (io == 1) words_to_bytes(span_ptr(msg, i), kv, 32);
  }
  if (hash) {
    uint32_t h[16];
    load_words(h, row, kWordH, 16);
    b2::mix_hash32(h, kv);
    store_words(row, kWordH, h, 16);
  }
  if (key) mix_key(row, kv, 32);
}

// ee / es / se / ss: MixKey(DH(key[sk], key[pk]))
__global__ __launch_bounds__(64) void k_hs_dh(HsSession *S, uint64_t n, int sk, int pk) {
  NOISE_HS_ROW();
  uint32_t a[8], b[8], shared[8];
  load_key(a, row, sk);
  load_key(b, row, pk);
  x25519::scalarmult(shared, a, b);
  mix_key(row, shared, 32);
}

// psk: MixKeyAndHash(psks[i][idx]): (ck, th, tk) = HKDF(ck, psk, 3);
// MixHash(th); k = tk[0..32)   (rev34 §5.2)
__global__ __launch_bounds__(64) void k_hs_psk(HsSession *S, uint64_t n, const uint8_t *psks,
                                               uint32_t npsk, uint32_t idx) {
  NOISE_HS_ROW();
  uint32_t psk[8], ck[16], o1[16], o2[16], o3[16], h[16];
  bytes_to_words(psk, psks + (i * npsk + idx) * 32, 32);
  load_words(ck, row, kWordCk, 16);
  b2::hkdf(ck, psk, 32, 3, o1, o2, o3);
  store_words(row, kWordCk, o1, 16);
  load_words(h, row, kWordH, 16);
  b2::mix_hash64(h, o2);
  store_words(row, kWordH, h, 16);
  store_words(row, kWordK, o3, 8);
}

// Message length check before a read: cursor_min <= len_i <= 65535, else the
// session fails with NOISE_GPU_HS_BAD_LEN.
// message length len[i] + add outside [min_len, 65535]: the session fails
// (read: len = message lengths, add 0; write: len = payload lengths, add =
// the message's fixed bytes, so no oversized message is ever written)
__global__ __launch_bounds__(64) void k_hs_check_len(HsSession *S, uint64_t n, const uint32_t *len,
                                                     uint32_t min_len, uint32_t add) {
  NOISE_HS_ROW();
  const uint64_t m = (uint64_t)len[i] + add;
  if (m < min_len || m > 65535u) fail(row, NOISE_GPU_HS_BAD_LEN);
}

// EncryptAndHash(src) -> dst: ct = ENCRYPT(k, nonce, h, pt) if has_k else pt;
// MixHash(ct).  src: key[src_key] (the "s" token, 32 B) or the payload span.
// out_len (optional): dst_cursor + bytes written, the message length.
__global__ __launch_bounds__(64) void k_hs_encrypt_hash(HsSession *S, uint64_t n, int has_k,
                                                        uint64_t nonce, int src_key, HsSpan src,
                                                        HsSpan dst, uint32_t *out_len) {
  NOISE_HS_ROW();
  uint8_t *out = span_ptr(dst, i);
  uint32_t kv[8];
  const uint8_t *in;
  int64_t len;
  if (src_key >= 0) {
    in = reinterpret_cast<const uint8_t *>(row) + 4 * (kWordKeys + 8 * src_key);
    len = 32;
  } else {
    in = span_ptr(src, i);
    len = span_len(src, i);
  }
  if (has_k) {
    load_words(kv, row, kWordK, 8);
    aead_record<false, false>(kv, nonce, in, out, (uint32_t)len,
                              reinterpret_cast<const uint8_t *>(row) + 4 * kWordH, 64);
    len += 16;
  } else {
    copy_bytes(out, in, len);
  }
  uint32_t h[16];
  load_words(h, row, kWordH, 16);
  b2::mix_hash_mem(h, out, len);
  store_words(row, kWordH, h, 16);
  if (out_len) out_len[i] = dst.add + (uint32_t)len;
}

// DecryptAndHash(src) -> dst: pt = DECRYPT(k, nonce, h, ct) if has_k else ct;
// MixHash(ct).  src: the message span (ct, with its tag when has_k); dst:
// key[dst_key] (the "s" token) or the payload span.  A bad tag fails the
// session (NOISE_GPU_HS_BAD_MAC) and zeroes the plaintext.
__global__ __launch_bounds__(64) void k_hs_decrypt_hash(HsSession *S, uint64_t n, int has_k,
                                                        uint64_t nonce, HsSpan src, int dst_key,
                                                        HsSpan dst, uint32_t *out_len) {
  NOISE_HS_ROW();
  const uint8_t *in = span_ptr(src, i);
  const int64_t ct_len = span_len(src, i);
  uint8_t *out = dst_key >= 0 ? reinterpret_cast<uint8_t *>(row) + 4 * (kWordKeys + 8 * dst_key)
                              : span_ptr(dst, i);
  const int64_t pt_len = has_k ? ct_len - 16 : ct_len;
  bool ok = true;
  if (has_k) {
    uint32_t kv[8];
    load_words(kv, row, kWordK, 8);
    ok = aead_record<true, false>(kv, nonce, in, out, (uint32_t)pt_len,
                                  reinterpret_cast<const uint8_t *>(row) + 4 * kWordH, 64);
  } else {
    copy_bytes(out, in, ct_len);
  }
  uint32_t h[16];
  load_words(h, row, kWordH, 16);
  b2::mix_hash_mem(h, in, ct_len);
  store_words(row, kWordH, h, 16);
  if (out_len) out_len[i] = ok ? (uint32_t)pt_len : 0u;
  if (!ok) fail(row, NOISE_GPU_HS_BAD_MAC);
}

// Split(): (t1, t2) = HKDF(ck, empty, 2) -> k1[i], k2[i] (32 B rows), and
// optionally the handshake hash h (64 B rows) and the remote static key.
// A failed session gets all-zero keys.
__global__ __launch_bounds__(64) void k_hs_split(HsSession *S, uint64_t n, uint8_t *k1,
                                                 uint8_t *k2, uint8_t *hash, uint8_t *rs) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  HsSession *row = S + i;
  uint32_t o1[16], o2[16], o3[16];
  if (live(row)) {
    uint32_t ck[16], none[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    load_words(ck, row, kWordCk, 16);
    b2::hkdf(ck, none, 0, 2, o1, o2, o3);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) o1[j] = o2[j] = 0u;
  }
  u32x4 *d1 = reinterpret_cast<u32x4 *>(k1 + 32 * i), *d2 = reinterpret_cast<u32x4 *>(k2 + 32 * i);
  d1[0] = u32x4{o1[0], o1[1], o1[2], o1[3]};
  d1[1] = u32x4{o1[4], o1[5], o1[6], o1[7]};
  d2[0] = u32x4{o2[0], o2[1], o2[2], o2[3]};
  d2[1] = u32x4{o2[4], o2[5], o2[6], o2[7]};
  if (hash) {
    uint32_t h[16];
    load_words(h, row, kWordH, 16);
    u32x4 *dh = reinterpret_cast<u32x4 *>(hash + 64 * i);
#pragma unroll
    for (int q = 0; q < 4; ++q) dh[q] = u32x4{h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]};
  }
  if (rs) {
    uint32_t r[8];
    load_key(r, row, kHsRs);
    u32x4 *dr = reinterpret_cast<u32x4 *>(rs + 32 * i);
    dr[0] = u32x4{r[0], r[1], r[2], r[3]};
    dr[1] = u32x4{r[4], r[5], r[6], r[7]};
  }
}

__global__ __launch_bounds__(64) void k_hs_status(const HsSession *S, uint64_t n, uint8_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  out[i] = (uint8_t)reinterpret_cast<const uint32_t *>(S + i)[kWordStatus];
}

// Wipe every row (keys, ck, h) before the batch is freed.
__global__ __launch_bounds__(64) void k_hs_wipe(HsSession *S, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  u32x4 *p = reinterpret_cast<u32x4 *>(S + i);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(HsSession) / 16); ++q) p[q] = u32x4{0, 0, 0, 0};
}

// ---- launchers -------------------------------------------------------------
namespace {
inline dim3 grid_of(uint64_t n) { return dim3((unsigned)((n + 63) / 64)); }
}  // namespace

hipError_t launch_hs_init(HsSession *S, uint64_t n, const HsWords16 &h0, const HsSpan &prologue,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_hs_init, grid_of(n), dim3(64), 0, st, S, n, h0, prologue);
  return hipGetLastError();
}
hipError_t launch_hs_set_key(HsSession *S, uint64_t n, int which, const uint8_t *src,
                             uint64_t src_stride, const HsWords8 &seed, uint32_t drbg_ctr,
                             bool derive_pk, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_set_key, grid_of(n), dim3(64), 0, st, S, n, which, src, src_stride, seed,
                     drbg_ctr, (int)derive_pk);
  return hipGetLastError();
}
hipError_t launch_hs_bcast_key(HsSession *S, uint64_t n, int which, int count, hipStream_t st) {
  if (n < 2) return hipSuccess;
  hipLaunchKernelGGL(k_hs_bcast_key, grid_of(n), dim3(64), 0, st, S, n, which, count);
  return hipGetLastError();
}
hipError_t launch_hs_key_token(HsSession *S, uint64_t n, int which, int io, const HsSpan &msg,
                               bool hash, bool key, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_key_token, grid_of(n), dim3(64), 0, st, S, n, which, io, msg, (int)hash,
                     (int)key);
  return hipGetLastError();
}
hipError_t launch_hs_dh(HsSession *S, uint64_t n, int sk, int pk, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_dh, grid_of(n), dim3(64), 0, st, S, n, sk, pk);
  return hipGetLastError();
}
hipError_t launch_hs_psk(HsSession *S, uint64_t n, const uint8_t *psks, uint32_t npsk,
                         uint32_t idx, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_psk, grid_of(n), dim3(64), 0, st, S, n, psks, npsk, idx);
  return hipGetLastError();
}
hipError_t launch_hs_check_len(HsSession *S, uint64_t n, const uint32_t *len, uint32_t min_len,
                               uint32_t add, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_check_len, grid_of(n), dim3(64), 0, st, S, n, len, min_len, add);
  return hipGetLastError();
}
hipError_t launch_hs_encrypt_hash(HsSession *S, uint64_t n, bool has_k, uint64_t nonce,
                                  int src_key, const HsSpan &src, const HsSpan &dst,
                                  uint32_t *out_len, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_encrypt_hash, grid_of(n), dim3(64), 0, st, S, n, (int)has_k, nonce,
                     src_key, src, dst, out_len);
  return hipGetLastError();
}
hipError_t launch_hs_decrypt_hash(HsSession *S, uint64_t n, bool has_k, uint64_t nonce,
                                  const HsSpan &src, int dst_key, const HsSpan &dst,
                                  uint32_t *out_len, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_decrypt_hash, grid_of(n), dim3(64), 0, st, S, n, (int)has_k, nonce, src,
                     dst_key, dst, out_len);
  return hipGetLastError();
}
hipError_t launch_hs_split(HsSession *S, uint64_t n, uint8_t *k1, uint8_t *k2, uint8_t *hash,
                           uint8_t *rs, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_split, grid_of(n), dim3(64), 0, st, S, n, k1, k2, hash, rs);
  return hipGetLastError();
}
hipError_t launch_hs_status(const HsSession *S, uint64_t n, uint8_t *out, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_status, grid_of(n), dim3(64), 0, st, S, n, out);
  return hipGetLastError();
}
hipError_t launch_hs_wipe(HsSession *S, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_hs_wipe, grid_of(n), dim3(64), 0, st, S, n);
  return hipGetLastError();
}

}  // namespace noise_amd
