// launchers.hpp -- internal interface between the C-ABI layer
// (noise_gpu_api.hip) and the kernels (aead_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "noise_gpu.h"

namespace noise_amd {

hipError_t launch_aead_uniform(bool decrypt, const uint32_t key[8],
                               uint64_t nonce0, const uint8_t *in,
                               uint64_t in_stride, uint8_t *out,
                               uint64_t out_stride, uint32_t len,
                               const uint8_t *ad, uint64_t ad_stride,
                               uint32_t ad_len, uint8_t *status, uint64_t nrec,
                               hipStream_t stream);

// len_sum: the records' plaintext bytes (0 = unknown): a batch below the
// classifier's record count whose records average >= 2 KiB is classified
// anyway (one lane walking a 16 KiB record costs more than the classifier)
hipError_t launch_aead_records(bool decrypt, const uint8_t *keys,
                               uint32_t nkeys, const noise_gpu_record *recs,
                               uint64_t nrec, const uint8_t *in, uint8_t *out,
                               const uint8_t *ad, uint8_t *status,
                               hipStream_t stream, uint64_t len_sum = 0);

// zero the records-path scratch of (current device, stream)
hipError_t records_scratch_wipe(hipStream_t stream);
// the grow-only scratch of (current device, stream), >= bytes; the records
// path and the uniform path's staging of unaligned batches share it
hipError_t records_scratch_get(void **p, size_t bytes, hipStream_t stream);
// zero + free the scratch and destroy the companion stream cached for
// (current device, stream); call before destroying `stream`
hipError_t records_scratch_release(hipStream_t stream);

bool sessions_supported(uint32_t len, const void *in, uint64_t in_stride,
                        const void *out, uint64_t out_stride);

hipError_t launch_aead_sessions(bool decrypt, const uint8_t *keys,
                                uint32_t nkeys, const uint32_t *key_idx,
                                const uint64_t *nonces, const uint8_t *in,
                                uint64_t in_stride, uint8_t *out,
                                uint64_t out_stride, uint32_t len,
                                uint8_t *status, uint64_t nrec,
                                hipStream_t stream);

hipError_t launch_rekey(uint8_t *keys, uint64_t nkeys, hipStream_t stream);

// ---- latency path (single_kernels.hip): one record per launch, staged in
// host-mapped pinned memory that the kernel reads and writes directly.
constexpr uint32_t kOneMaxAd = 8192;  // larger AD takes the copy-staged path
struct OneLayout {
  uint64_t ad, in, tag, out, total;
};
// Host image (host-mapped pinned):
// [0,64) done line, GPU -> host (u32 done word, u32 status, u32 alive)
// [64,128) OneRing: the resident kernel's stop word, host -> GPU
// then AD | record | tag (the launch path's input) | output
constexpr uint32_t kOneRingOff = 64;
struct OneRing {
  uint64_t pad0;
  uint32_t stop;      // nonzero: the resident kernel exits
  uint32_t pad1[13];
};
static_assert(sizeof(OneRing) == 64, "stop line");
// Resident request image (OneReq; device memory the host writes through the
// BAR, or host-mapped): kReqChunks 16-byte chunks, each {seq, w1, w2, w3},
// that the kernel polls:
//   chunk 0: seq, len | ad_len << 16 | decrypt << 30, nonce lo, nonce hi
//   chunk 1: seq, key words 0, 1, 2      chunk 2: seq, key words 3, 4, 5
//   chunk 3: seq, key words 6, 7, check word (req_check_word)
//   chunks 4 ..: a small record INLINE -- its staged image (AD | pad |
//     record | pad | tag, the 16-byte pieces the kernel works on) 12 bytes
//     per chunk, so every chunk carries the seq that validates it and the
//     record arrives with the poll that finds the request (req_inline)
// then, at kReqStageOff, a larger record's AD | record | tag at one_layout()
// offsets, loaded by DMA once the request is seen.  Output goes to the host
// image.  The kernel zeroes the request after use (but for the header
// chunks' seq words).
constexpr uint32_t kReqChunks = 128;
constexpr uint32_t kReqInlineBytes = 12u * (kReqChunks - 4u);  // 1488
constexpr uint64_t kReqStageOff = 16ull * kReqChunks;
__host__ __device__ constexpr uint32_t req_image_bytes(uint32_t ad_len, uint32_t len, bool decrypt) {
  return 16u * (((ad_len + 15u) >> 4) + ((len + 15u) >> 4) + (decrypt ? 1u : 0u));
}
__host__ __device__ constexpr bool req_inline(uint32_t ad_len, uint32_t len, bool decrypt) {
  return req_image_bytes(ad_len, len, decrypt) <= kReqInlineBytes;
}
__host__ __device__ constexpr uint32_t req_inline_chunks(uint32_t ad_len, uint32_t len, bool decrypt) {
  return req_inline(ad_len, len, decrypt) ? (req_image_bytes(ad_len, len, decrypt) + 11u) / 12u : 0u;
}
// Every chunk of a request carries its own check: its first word is
// seq ^ req_chunk_tag(chunk, w1, w2, w3) over its three payload words.  The
// kernel decodes each chunk it polls and takes a request only when the four
// header chunks (and every inline chunk) decode to the same new seq, so a
// chunk whose 16-byte BAR store landed in part (new first word, stale
// payload, or the reverse) decodes to something else and is polled again.
// The check is per lane, folded into the seq compare (round 5): round 4's
// single check word needed a cross-lane sum on the accept path.  The chunk
// constant keeps an all-zero image (never a request) from decoding to one
// seq in all four header chunks.  The tag is non-linear (round 6, ADVICE
// r5): the words are multiplied by odd constants before they are combined
// and the sum goes through a multiply / xorshift finaliser, so a tear that
// leaves stale (e.g. wiped, zero) payload words under a new seq word does
// not decode to that seq for structured payloads the way XOR-of-rotations
// did (len 64 with nonce 2^26 cancelled exactly: rotl(64, 7) == rotl(2^26,
// 19)).  tests/cpp/req_tag_test.cpp tears chunk 0 over small meta / nonces.
__host__ __device__ constexpr uint32_t req_rotl(uint32_t x, int n) {
  return (x << n) | (x >> (32 - n));
}
__host__ __device__ constexpr uint32_t req_chunk_tag(uint32_t chunk, uint32_t w1, uint32_t w2,
                                                     uint32_t w3) {
  uint32_t x = w1 * 0x9e3779b1u + (chunk + 1u) * 0x7f4a7c15u;
  x ^= req_rotl(w2 * 0x85ebca6bu, 13);
  x ^= req_rotl(w3 * 0xc2b2ae35u, 17);
  x *= 0x27d4eb2fu;
  return x ^ (x >> 15);
}
__host__ __device__ constexpr OneLayout one_layout(uint32_t ad_len, uint32_t len) {
  const uint64_t a16 = (ad_len + 15ull) & ~15ull, l16 = (len + 15ull) & ~15ull;
  OneLayout o{};
  o.ad = 128;
  o.in = o.ad + a16;
  o.tag = o.in + l16;
  o.out = o.tag + 16;
  o.total = o.out + l16 + 16;
  return o;
}
constexpr uint64_t kOneReqBytes = kReqStageOff + one_layout(kOneMaxAd, 65535u).total;
// the resident kernel's records: <= 63 keystream blocks (its quad path)
constexpr uint32_t kResidentMaxLen = 63u * 64u;
// dynamic LDS of the latency kernels: staged pieces + tag, r, s, verdict and
// the per-wave Poly1305 sums
__host__ __device__ constexpr size_t one_lds_bytes(uint32_t ad_len, uint32_t len) {
  return 16ull * (((ad_len + 15u) >> 4) + ((len + 15u) >> 4) + 4u + 8u);
}
hipError_t launch_aead_one(bool decrypt, const uint32_t key[8], uint64_t nonce,
                           uint8_t *d_base, uint32_t len, uint32_t ad_len, uint32_t seq,
                           hipStream_t stream);
// the resident latency kernel: requests from the image at d_req (OneReq),
// output and done word in the host image at d_base (both sized for
// one_layout(kOneMaxAd, 65535)); `last` = the seq already served
hipError_t launch_aead_resident(uint8_t *d_req, uint8_t *d_base, uint32_t last, uint32_t idle_us,
                                hipStream_t stream);

hipError_t launch_x25519(const uint8_t *scalars, const uint8_t *points,
                         uint8_t *out, uint64_t n, hipStream_t stream);

// ---- batched handshakes (handshake_kernels.hip, handshake_batch.hip) ----
// One session's handshake state in HBM (AoS row, 16-byte aligned words).
struct HsSession {
  uint32_t ck[16];      // chaining key
  uint32_t h[16];       // handshake hash
  uint32_t k[8];        // CipherState key (meaningful while the host's has_k)
  uint32_t status;      // 0, or the sticky NOISE_GPU_HS_* failure code
  uint32_t pad[7];
  uint32_t keys[6][8];  // HsKey slots
};
enum HsKey : int { kHsSsk = 0, kHsSpk = 1, kHsEsk = 2, kHsEpk = 3, kHsRs = 4, kHsRe = 5 };
struct HsWords16 { uint32_t w[16]; };
struct HsWords8 { uint32_t w[8]; };
// Per-session byte range: base + (off ? off[i] : i * stride) + add, length
// len ? len[i] + len_adj : len_u.
struct HsSpan {
  uint8_t *base;
  const uint64_t *off;
  uint64_t stride;
  const uint32_t *len;
  uint32_t len_u;
  int32_t len_adj;
  uint32_t add;
  uint32_t pad;
};

hipError_t launch_hs_init(HsSession *S, uint64_t n, const HsWords16 &h0, const HsSpan &prologue,
                          hipStream_t st);
hipError_t launch_hs_set_key(HsSession *S, uint64_t n, int which, const uint8_t *src,
                             uint64_t src_stride, const HsWords8 &seed, uint32_t drbg_ctr,
                             bool derive_pk, hipStream_t st);
hipError_t launch_hs_bcast_key(HsSession *S, uint64_t n, int which, int count, hipStream_t st);
hipError_t launch_hs_key_token(HsSession *S, uint64_t n, int which, int io, const HsSpan &msg,
                               bool hash, bool key, hipStream_t st);
hipError_t launch_hs_dh(HsSession *S, uint64_t n, int sk, int pk, hipStream_t st);
hipError_t launch_hs_psk(HsSession *S, uint64_t n, const uint8_t *psks, uint32_t npsk,
                         uint32_t idx, hipStream_t st);
hipError_t launch_hs_check_len(HsSession *S, uint64_t n, const uint32_t *len, uint32_t min_len,
                               uint32_t add, hipStream_t st);
hipError_t launch_hs_encrypt_hash(HsSession *S, uint64_t n, bool has_k, uint64_t nonce,
                                  int src_key, const HsSpan &src, const HsSpan &dst,
                                  uint32_t *out_len, hipStream_t st);
hipError_t launch_hs_decrypt_hash(HsSession *S, uint64_t n, bool has_k, uint64_t nonce,
                                  const HsSpan &src, int dst_key, const HsSpan &dst,
                                  uint32_t *out_len, hipStream_t st);
hipError_t launch_hs_split(HsSession *S, uint64_t n, uint8_t *k1, uint8_t *k2, uint8_t *hash,
                           uint8_t *rs, hipStream_t st);
hipError_t launch_hs_status(const HsSession *S, uint64_t n, uint8_t *out, hipStream_t st);
hipError_t launch_hs_wipe(HsSession *S, uint64_t n, hipStream_t st);

// C-ABI helpers shared by the API translation units (noise_gpu_api.hip)
int api_hip_fail(hipError_t e, const char *what);
int api_arg_fail(const char *msg);
int api_check_device();

hipError_t launch_fill_synthetic(uint8_t *dst, uint64_t offset,
                                 uint64_t nbytes, uint64_t seed,
                                 hipStream_t stream);

}  // namespace noise_amd
