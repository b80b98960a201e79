// aead_kernels.hip -- gfx950 kernels of the Noise ChaChaPoly record engine
// and their host-side launchers (called by noise_gpu_api.hip).
//
//   k_encrypt_uniform / k_decrypt_uniform   one key, fixed length, implicit
//                                            nonce0 + i, fixed strides (the
//                                            BASELINE config-2 hot path)
//   (descriptor batches: records_kernels.hip)
//   k_rekey                                  CipherState::rekey on a table
//   k_fill_synthetic                         splitmix64 test/bench data
//
// One lane = one record (chachapoly_device.hpp).  Launch: 256-thread
// workgroups, one record per thread; the grid covers nrec.
#include "chachapoly_device.hpp"
#include "launchers.hpp"
#include "mtile_kernel.hpp"
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kBlock = 256;

template <bool DECRYPT, bool VEC>
__global__ __launch_bounds__(kBlock) void k_aead_uniform(
    KeyArg key, uint64_t nonce0, const uint8_t *__restrict__ in,
    uint64_t in_stride, uint8_t *out, uint64_t out_stride, uint32_t len,
    const uint8_t *ad, uint64_t ad_stride, uint32_t ad_len, uint8_t *status,
    uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nrec) return;
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = key.w[j];
  const bool ok = aead_record<DECRYPT, VEC>(
      k, nonce0 + i, in + i * in_stride, out + i * out_stride, len,
      ad + i * ad_stride, ad_len);
  if (DECRYPT) status[i] = ok ? 0u : 1u;
}

// REKEY: k <- ENCRYPT(k, 2^64-2, empty, 0^32)[0..32) = first 32 keystream
// bytes of block 1 at nonce 2^64-2 (the zero plaintext makes ct = ks).
__global__ __launch_bounds__(kBlock) void k_rekey(uint8_t *keys, uint64_t nkeys) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nkeys) return;
  uint4 *kp = reinterpret_cast<uint4 *>(keys + 32u * i);
  const uint4 ka = kp[0], kb = kp[1];
  const uint32_t k[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
  const uint64_t n = ~0ull - 1ull;
  uint32_t ks[16];
  chacha20_block(k, 1u, (uint32_t)n, (uint32_t)(n >> 32), ks);
  kp[0] = make_uint4(ks[0], ks[1], ks[2], ks[3]);
  kp[1] = make_uint4(ks[4], ks[5], ks[6], ks[7]);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// 16 bytes per thread; `offset` and d_dst 16-byte aligned on this path.
__global__ __launch_bounds__(kBlock) void k_fill_synthetic_vec(
    uint4 *dst, uint64_t offset, uint64_t nvec, uint64_t seed) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nvec) return;
  const uint64_t w = (offset >> 3) + 2 * i;
  const uint64_t a = mix64(seed + (w + 1) * 0x9e3779b97f4a7c15ull);
  const uint64_t b = mix64(seed + (w + 2) * 0x9e3779b97f4a7c15ull);
  dst[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b,
                      (uint32_t)(b >> 32));
}

__global__ __launch_bounds__(kBlock) void k_fill_synthetic_bytes(
    uint8_t *dst, uint64_t offset, uint64_t nbytes, uint64_t seed) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= nbytes) return;
  const uint64_t b = offset + j;
  dst[j] = (uint8_t)(mix64(seed + ((b >> 3) + 1) * 0x9e3779b97f4a7c15ull) >>
                     (8 * (b & 7)));
}

static inline dim3 grid_for(uint64_t n) {
  return dim3((unsigned)((n + kBlock - 1) / kBlock));
}

// ---- unaligned uniform batches, staged --------------------------------------
// Records that do not start 16-byte aligned (the Noise wire format packed back
// to back with a length that is not a multiple of 16: 1000-byte records at
// strides 1000 / 1016) cannot be LDS-DMA'd piece by piece.  They are copied
// into an aligned image in the scratch (row stride ceil16(len + 16)), the
// tile kernels run on it in place, and the outputs are copied back.  The two
// copies are HBM-bound passes beside a VALU-bound kernel.
//
// k_stage_in: thread (record i, piece p) moves source bytes [16p, 16p + 16) of
// record i (n bytes) to the aligned row: two aligned loads and a byte funnel
// (a 16-byte aligned block holding a byte of the record never crosses a
// page); bytes past n are don't-care (the tile kernels mask them).
__global__ __launch_bounds__(kBlock) void k_stage_in(const uint8_t *in, uint64_t in_stride,
                                                     uint8_t *s, uint64_t sstride, uint32_t n,
                                                     uint32_t np, uint64_t nrec) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t i = t / np;
  const uint32_t p = (uint32_t)(t % np);
  if (i >= nrec) return;
  const uintptr_t a = reinterpret_cast<uintptr_t>(in + i * in_stride) + 16ull * p;
  const uint32_t sh = (uint32_t)(a & 15u);
  const uint4 *b = reinterpret_cast<const uint4 *>(a - sh);
  const uint32_t have = n - 16u * p < 16u ? n - 16u * p : 16u;  // this piece's record bytes
  uint4 v = b[0];
  if (sh) {
    const uint4 hi = sh + have > 16u ? b[1] : make_uint4(0u, 0u, 0u, 0u);
    v = extract16(v, hi, sh);
  }
  *reinterpret_cast<uint4 *>(s + i * sstride + 16ull * p) = v;
}

// k_stage_out: thread (record i, block b) writes the 16-byte aligned block b of
// record i's destination range [D, D + n) (blocks from floor16(D)), only the
// record's own bytes: whole blocks by one 16-byte store, the partial first and
// last blocks byte by byte (a neighbouring record may own the rest).  Decrypt:
// a record whose tag failed is skipped (in place: left as it was) or zeroed.
__global__ __launch_bounds__(kBlock) void k_stage_out(const uint8_t *s, uint64_t sstride,
                                                      uint8_t *out, uint64_t out_stride, uint32_t n,
                                                      uint32_t nb, const uint8_t *status,
                                                      int keep_failed, uint64_t nrec) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t i = t / nb;
  const uint32_t bi = (uint32_t)(t % nb);
  if (i >= nrec) return;
  const uintptr_t d = reinterpret_cast<uintptr_t>(out + i * out_stride);
  const uintptr_t blk = (d & ~(uintptr_t)15u) + 16ull * bi;
  const uintptr_t lo = blk > d ? blk : d, hi = blk + 16u < d + n ? blk + 16u : d + n;
  if (lo >= hi) return;
  bool zero = false;
  if (status && status[i] != 0u) {
    if (keep_failed) return;
    zero = true;
  }
  // byte k of the block = staged byte off + k of the record
  const int64_t off = (int64_t)blk - (int64_t)d;  // >= -15
  const int64_t a0 = off >= 0 ? (off & ~(int64_t)15) : -16;
  const uint32_t sh = (uint32_t)(off - a0);
  const uint8_t *row = s + i * sstride;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  const uint4 A = a0 >= 0 ? *reinterpret_cast<const uint4 *>(row + a0) : z;
  const uint4 B = (sh && a0 + 16 < (int64_t)sstride) ? *reinterpret_cast<const uint4 *>(row + a0 + 16) : z;
  uint4 v = sh ? extract16(A, B, sh) : A;
  if (zero) v = z;
  uint8_t *bp = reinterpret_cast<uint8_t *>(blk);
  if (lo == blk && hi == blk + 16u) {
    store16<true>(bp, v, 16);
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t j = (uint32_t)(lo - blk); j < (uint32_t)(hi - blk); ++j)
      bp[j] = (uint8_t)(w[j >> 2] >> (8u * (j & 3u)));
  }
}

// records per call from which staging beats the lane walk; scratch per slice
constexpr uint64_t kStageMin = 1024;
#ifndef NOISE_STAGE_BYTES
#define NOISE_STAGE_BYTES (1ull << 30)
#endif
constexpr uint64_t kStageBytes = NOISE_STAGE_BYTES;

hipError_t launch_aead_uniform(bool decrypt, const uint32_t key[8],
                               uint64_t nonce0, const uint8_t *in,
                               uint64_t in_stride, uint8_t *out,
                               uint64_t out_stride, uint32_t len,
                               const uint8_t *ad, uint64_t ad_stride,
                               uint32_t ad_len, uint8_t *status, uint64_t nrec,
                               hipStream_t stream) {
  if (nrec == 0) return hipSuccess;
  KeyArg k;
  for (int j = 0; j < 8; ++j) k.w[j] = key[j];
  const bool vec = ((reinterpret_cast<uintptr_t>(in) |
                     reinterpret_cast<uintptr_t>(out) | in_stride |
                     out_stride | len) & 15u) == 0;
  // LDS-staged tile kernel: aligned, AD-free, supported lengths
  if (vec && ad_len == 0) {
    TileArgs ta{};
    ta.key = k;
    ta.nonce0 = nonce0;
    ta.in = in;
    ta.in_stride = in_stride;
    ta.out = out;
    ta.out_stride = out_stride;
    ta.status = status;
    ta.nrec = nrec;
    ta.in_place = in == out;
    const dim3 gt((unsigned)((nrec + 63) / 64)), bt(64);
    // packed records (stride == record size on both sides): cheap addressing
    const bool contig = decrypt ? (in_stride == (uint64_t)len + 16 && out_stride == len)
                                : (in_stride == len && out_stride == (uint64_t)len + 16);
#ifndef NOISE_UNIFORM_SPAN  // bytes per lane of the uniform tile kernels (A/B: 128)
#define NOISE_UNIFORM_SPAN 256
#endif
#define NOISE_TILE_LAUNCH(DEC, LEN, CONTIG)                                    \
    hipLaunchKernelGGL((k_aead_tile<DEC, LEN, CONTIG, kTileUniform, 0, 1,       \
                                    (LEN >= 256 && LEN <= 8192) ? NOISE_UNIFORM_SPAN : 256>), \
                       gt, bt, 0, stream, ta)
#define NOISE_TILE_CASE(LEN)                                                   \
    case LEN:                                                                  \
      if (decrypt) {                                                           \
        if (contig) NOISE_TILE_LAUNCH(true, LEN, true);                        \
        else NOISE_TILE_LAUNCH(true, LEN, false);                              \
      } else {                                                                 \
        if (contig) NOISE_TILE_LAUNCH(false, LEN, true);                       \
        else NOISE_TILE_LAUNCH(false, LEN, false);                             \
      }                                                                        \
      return hipGetLastError();
    switch (len) {
      NOISE_TILE_CASE(64)
      NOISE_TILE_CASE(128)
      NOISE_TILE_CASE(192)
      NOISE_TILE_CASE(256)
      NOISE_TILE_CASE(512)
      NOISE_TILE_CASE(1024)
      NOISE_TILE_CASE(2048)
      NOISE_TILE_CASE(4096)
      NOISE_TILE_CASE(8192)
      NOISE_TILE_CASE(16384)
      default: break;
    }
#undef NOISE_TILE_CASE
#undef NOISE_TILE_LAUNCH
  }
  // any other length up to 16 KiB with 16-byte aligned bases and strides:
  // the masked tile kernel at the smallest tile capacity >= len
  // (mtile_kernel.hpp).  Capacities between the
  // powers of two: one lane of 5 .. 7 chunks per record (320 .. 448 B), or
  // G = 3, 5, 6, 7, 9, 10, 12, 20 lanes of 4 chunks with 60-63 of 64 lanes
  // working.  The cost of a record ~ capacity x 64 / working lanes rises with
  // the capacity along this list, so the smallest that holds len is the
  // cheapest.  (Not listed: 3840, 5376, 7680 -- they idle enough lanes to
  // cost as much as the next power of two -- and nothing between 8 and 16 KiB,
  // where a tile holds one record and the idle lanes would be 1/8 .. 1/2.)
  const bool al = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out) | in_stride |
                    out_stride) & 15u) == 0;
  if (al && ad_len == 0 && len >= 1 && len <= 16384) {
    TileArgs ta{};
    ta.key = k;
    ta.nonce0 = nonce0;
    ta.in = in;
    ta.in_stride = in_stride;
    ta.out = out;
    ta.out_stride = out_stride;
    ta.status = status;
    ta.nrec = nrec;
    ta.in_place = in == out;
    ta.len = len;
    ta.chunk = -1;
#define NOISE_MTILE(LEN)                                                       \
    if (len <= LEN) {                                                          \
      constexpr uint64_t rps = MTileCfg<LEN>::RPS;                             \
      const dim3 gm((unsigned)((nrec + rps - 1) / rps)), bm(64);               \
      if (decrypt) hipLaunchKernelGGL((k_aead_mtile<true, LEN, kMTUniform>), gm, bm, 0, stream, ta); \
      else hipLaunchKernelGGL((k_aead_mtile<false, LEN, kMTUniform>), gm, bm, 0, stream, ta);        \
      return hipGetLastError();                                                \
    }
    NOISE_MTILE(64)
    NOISE_MTILE(128)
    NOISE_MTILE(192)
    NOISE_MTILE(256)
    NOISE_MTILE(320)
    NOISE_MTILE(384)
    NOISE_MTILE(448)
    NOISE_MTILE(512)
    NOISE_MTILE(768)
    NOISE_MTILE(1024)
    NOISE_MTILE(1280)
    NOISE_MTILE(1536)
    NOISE_MTILE(1792)
    NOISE_MTILE(2048)
    NOISE_MTILE(2304)
    NOISE_MTILE(2560)
    NOISE_MTILE(3072)
    NOISE_MTILE(4096)
    NOISE_MTILE(5120)
    NOISE_MTILE(8192)
    NOISE_MTILE(16384)
#undef NOISE_MTILE
  }
  // unaligned records up to 16 KiB, no AD: staged through an aligned image
  // (k_stage_in / k_stage_out above), the tile kernels in place on it
  const bool inplace = in == out && in_stride == out_stride;
  if (!al && ad_len == 0 && len >= 1 && len <= 16384 && nrec >= kStageMin &&
      (inplace || in + in_stride * nrec <= out || out + out_stride * nrec <= in)) {
    // in slices of at most kStageBytes of scratch (stream-ordered reuse)
    const uint64_t sstride = ((uint64_t)len + 31u) & ~15ull;
    const uint64_t per = kStageBytes / sstride > kStageMin ? kStageBytes / sstride : kStageMin;
    const uint64_t cap = nrec < per ? nrec : per;
    void *mem = nullptr;
    hipError_t e = records_scratch_get(&mem, cap * sstride, stream);
    if (e != hipSuccess) return e;
    uint8_t *s = static_cast<uint8_t *>(mem);
    const uint32_t nin = decrypt ? len + 16u : len, nout = decrypt ? len : len + 16u;
    const uint32_t np = (nin + 15u) / 16u, nb = nout / 16u + 2u;
    for (uint64_t r0 = 0; r0 < nrec; r0 += cap) {
      const uint64_t n = nrec - r0 < cap ? nrec - r0 : cap;
      hipLaunchKernelGGL(k_stage_in, grid_for(n * np), dim3(kBlock), 0, stream, in + r0 * in_stride, in_stride,
                         s, sstride, nin, np, n);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      e = launch_aead_uniform(decrypt, key, nonce0 + r0, s, sstride, s, sstride, len, nullptr, 0, 0,
                              status ? status + r0 : nullptr, n, stream);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_stage_out, grid_for(n * nb), dim3(kBlock), 0, stream, s, sstride,
                         out + r0 * out_stride, out_stride, nout, nb, decrypt ? status + r0 : nullptr,
                         inplace ? 1 : 0, n);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const dim3 g = grid_for(nrec), b(kBlock);
  if (decrypt) {
    if (vec)
      hipLaunchKernelGGL((k_aead_uniform<true, true>), g, b, 0, stream, k, nonce0, in, in_stride, out, out_stride, len, ad, ad_stride, ad_len, status, nrec);
    else
      hipLaunchKernelGGL((k_aead_uniform<true, false>), g, b, 0, stream, k, nonce0, in, in_stride, out, out_stride, len, ad, ad_stride, ad_len, status, nrec);
  } else {
    if (vec)
      hipLaunchKernelGGL((k_aead_uniform<false, true>), g, b, 0, stream, k, nonce0, in, in_stride, out, out_stride, len, ad, ad_stride, ad_len, status, nrec);
    else
      hipLaunchKernelGGL((k_aead_uniform<false, false>), g, b, 0, stream, k, nonce0, in, in_stride, out, out_stride, len, ad, ad_stride, ad_len, status, nrec);
  }
  return hipGetLastError();
}

hipError_t launch_rekey(uint8_t *keys, uint64_t nkeys, hipStream_t stream) {
  if (nkeys == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rekey, grid_for(nkeys), dim3(kBlock), 0, stream, keys, nkeys);
  return hipGetLastError();
}

hipError_t launch_fill_synthetic(uint8_t *dst, uint64_t offset,
                                 uint64_t nbytes, uint64_t seed,
                                 hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) | offset) & 15u) == 0;
  uint64_t head = 0;
  if (vec) {
    const uint64_t nvec = nbytes >> 4;
    if (nvec)
      hipLaunchKernelGGL(k_fill_synthetic_vec, grid_for(nvec), dim3(kBlock), 0, stream,
                         reinterpret_cast<uint4 *>(dst), offset, nvec, seed);
    head = nvec << 4;
  }
  if (head < nbytes)
    hipLaunchKernelGGL(k_fill_synthetic_bytes, grid_for(nbytes - head), dim3(kBlock), 0,
                       stream, dst + head, offset + head, nbytes - head, seed);
  return hipGetLastError();
}

}  // namespace noise_amd
