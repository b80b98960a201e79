// records_kernels.hip -- descriptor batches (noise_gpu_{en,de}crypt_records):
// many sessions, mixed sizes (BASELINE config 4, the wavefront load-balance
// study).
//
// A batch of arbitrary records is load-balanced by CLASS, entirely on the
// device and stream-ordered (no host round trip):
//   1. k_class_count / k_class_scatter: a counting sort of descriptor
//      indices by class, wave-aggregated atomics (one atomic per wave and
//      class);
//   2. one launch per class, each reading its slice and count from device
//      memory (capped grids that stride or pull work, so an empty class
//      costs one tiny launch):
//        - tile classes: 16-byte aligned, AD-free records of length
//          64, 128, 192, 256, 512, 1 Ki, 2 Ki, 4 Ki, 8 Ki, 16 Ki -> the
//          LDS-staged tile kernel (tile_kernel.hpp, kTileDesc), G lanes per
//          record;
//        - wave class: aligned, AD-free, longer than 16 KiB (any length,
//          e.g. 65519) -> one wavefront per record (wave_kernel.hpp);
//        - generic: everything else (AD, odd lengths <= 16 KiB, unaligned,
//          bad key index) -> one lane per record (chachapoly_device.hpp).
// Small batches (< kClassifyMin records) skip the sort and run the generic
// kernel directly (latency of single records from CipherState).
// Scratch (class counts + the sorted index array, 4 B per record) is a
// grow-only device buffer cached per (device, stream).
#include <mutex>
#include <vector>

#include "chachapoly_device.hpp"
#include "launchers.hpp"
#include "tile_kernel.hpp"
#include "wave_kernel.hpp"

namespace noise_amd {

constexpr int kGenBlock = 256;
constexpr int kNumTileCls = 10;
constexpr int kClsWave = kNumTileCls;
constexpr int kClsGeneric = kNumTileCls + 1;
constexpr int kNumCls = kNumTileCls + 2;
constexpr uint64_t kClassifyMin = 2048;
// Grid caps of the per-class launches (capped grids stride / pull work).
// 2048 single-wave workgroups = 8 per CU, what the register budget keeps
// resident.  Overridable for the CPU emulation build (tools/emu).
#ifndef NOISE_GRID_CAP
#define NOISE_GRID_CAP 2048u
#endif

__device__ __forceinline__ int tile_class(uint32_t len) {
  switch (len) {
    case 64: return 0;
    case 128: return 1;
    case 192: return 2;
    case 256: return 3;
    case 512: return 4;
    case 1024: return 5;
    case 2048: return 6;
    case 4096: return 7;
    case 8192: return 8;
    case 16384: return 9;
    default: return -1;
  }
}

__device__ __forceinline__ int record_class(const noise_gpu_record &d,
                                            uint32_t nkeys, const uint8_t *in,
                                            const uint8_t *out) {
  if (d.key_idx >= nkeys || d.ad_len != 0 || d.len == 0) return kClsGeneric;
  if (((reinterpret_cast<uintptr_t>(in + d.in_off) |
        reinterpret_cast<uintptr_t>(out + d.out_off)) & 15u) != 0)
    return kClsGeneric;
  const int t = tile_class(d.len);
  if (t >= 0) return t;
  return d.len > 16384u ? kClsWave : kClsGeneric;
}

// scratch layout (device): counts[kNumCls], cursors[kNumCls], wave cursor,
// then the sorted index array
struct RecScratch {
  unsigned long long counts[kNumCls];
  unsigned long long cursors[kNumCls];
  unsigned long long wave_cursor;
  unsigned long long pad[16 - ((2 * kNumCls + 1) % 16)];
};
static_assert(sizeof(RecScratch) % 128 == 0, "scratch header alignment");

__global__ __launch_bounds__(kGenBlock) void k_class_count(
    const noise_gpu_record *__restrict__ recs, uint64_t nrec, uint32_t nkeys,
    const uint8_t *in, const uint8_t *out, RecScratch *sc) {
  const uint64_t i = (uint64_t)blockIdx.x * kGenBlock + threadIdx.x;
  const int cls = i < nrec ? record_class(recs[i], nkeys, in, out) : -1;
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll 1
  for (int c = 0; c < kNumCls; ++c) {
    const uint64_t m = __ballot(cls == c);
    if (m != 0 && lane == (uint32_t)__builtin_ctzll(m))
      atomicAdd(&sc->counts[c], (unsigned long long)__builtin_popcountll(m));
  }
}

__global__ __launch_bounds__(kGenBlock) void k_class_scatter(
    const noise_gpu_record *__restrict__ recs, uint64_t nrec, uint32_t nkeys,
    const uint8_t *in, const uint8_t *out, RecScratch *sc, uint32_t *idx) {
  const uint64_t i = (uint64_t)blockIdx.x * kGenBlock + threadIdx.x;
  const int cls = i < nrec ? record_class(recs[i], nkeys, in, out) : -1;
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t base = 0;
#pragma unroll 1
  for (int c = 0; c < kNumCls; ++c) {
    const uint64_t m = __ballot(cls == c);
    if (m != 0) {
      const uint32_t leader = (uint32_t)__builtin_ctzll(m);
      unsigned long long old = 0;
      if (lane == leader)
        old = atomicAdd(&sc->cursors[c], (unsigned long long)__builtin_popcountll(m));
      old = ((unsigned long long)__shfl((int)(uint32_t)(old >> 32), leader) << 32) |
            (uint32_t)__shfl((int)(uint32_t)old, leader);
      if (cls == c) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        idx[base + old + rank] = (uint32_t)i;
      }
    }
    base += sc->counts[c];
  }
}

// one lane per record; idx == nullptr: record i directly (small batches)
template <bool DECRYPT>
__global__ __launch_bounds__(kGenBlock) void k_aead_records(
    const uint8_t *__restrict__ keys, uint32_t nkeys,
    const noise_gpu_record *__restrict__ recs, uint64_t nrec,
    const uint32_t *__restrict__ idx, const unsigned long long *counts,
    const uint8_t *in, uint8_t *out, const uint8_t *ad, uint8_t *status) {
  uint64_t base = 0, n = nrec;
  if (idx) {
    for (int c = 0; c < kClsGeneric; ++c) base += counts[c];
    n = counts[kClsGeneric];
  }
#pragma unroll 1
  for (uint64_t i = (uint64_t)blockIdx.x * kGenBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kGenBlock) {
    const uint64_t di = idx ? idx[base + i] : i;
    const noise_gpu_record r = recs[di];
    if (r.key_idx >= nkeys) {  // never index outside the key table
      if (DECRYPT) status[di] = NOISE_GPU_REC_BAD_KEY;
      continue;
    }
    const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 32u * r.key_idx);
    const uint4 ka = kp[0], kb = kp[1];
    const uint32_t k[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
    const uint8_t *src = in + r.in_off;
    uint8_t *dst = out + r.out_off;
    const bool vec = ((reinterpret_cast<uintptr_t>(src) |
                       reinterpret_cast<uintptr_t>(dst) | r.len) & 15u) == 0;
    bool ok;
    if (vec)
      ok = aead_record<DECRYPT, true>(k, r.nonce, src, dst, r.len, ad + r.ad_off, r.ad_len);
    else
      ok = aead_record<DECRYPT, false>(k, r.nonce, src, dst, r.len, ad + r.ad_off, r.ad_len);
    if (DECRYPT) status[di] = ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
  }
}

// ---- scratch: one grow-only buffer per (device, stream) ------------------
// Calls on one stream are ordered, so they may share the buffer; a buffer
// only grows (hipFree waits for the device, so a smaller one still in use by
// an earlier launch is never released under it).
static hipError_t scratch_get(void **p, size_t bytes, hipStream_t stream) {
  struct Entry {
    int dev;
    hipStream_t stream;
    void *ptr;
    size_t size;
  };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  for (Entry &en : cache) {
    if (en.dev != dev || en.stream != stream) continue;
    if (en.size < bytes) {
      if ((e = hipFree(en.ptr)) != hipSuccess) return e;
      en.ptr = nullptr;
      en.size = 0;
      if ((e = hipMalloc(&en.ptr, bytes)) != hipSuccess) return e;
      en.size = bytes;
    }
    *p = en.ptr;
    return hipSuccess;
  }
  void *ptr = nullptr;
  if ((e = hipMalloc(&ptr, bytes)) != hipSuccess) return e;
  cache.push_back({dev, stream, ptr, bytes});
  *p = ptr;
  return hipSuccess;
}

template <bool DECRYPT>
static void launch_desc_tiles(const TileArgs &ta, uint64_t nrec, hipStream_t stream) {
  const dim3 bt(64);
  auto grid = [&](int rpt_super) {
    (void)rpt_super;
    const uint64_t want = (nrec + 63) / 64;
    return dim3((unsigned)(want < NOISE_GRID_CAP ? want : NOISE_GRID_CAP));
  };
  TileArgs a = ta;
#define NOISE_DESC_TILE(C, LEN)                                                \
  a.cls = C;                                                                   \
  hipLaunchKernelGGL((k_aead_tile<DECRYPT, LEN, false, kTileDesc>), grid(LEN), bt, 0, stream, a);
  NOISE_DESC_TILE(0, 64)
  NOISE_DESC_TILE(1, 128)
  NOISE_DESC_TILE(2, 192)
  NOISE_DESC_TILE(3, 256)
  NOISE_DESC_TILE(4, 512)
  NOISE_DESC_TILE(5, 1024)
  NOISE_DESC_TILE(6, 2048)
  NOISE_DESC_TILE(7, 4096)
  NOISE_DESC_TILE(8, 8192)
  NOISE_DESC_TILE(9, 16384)
#undef NOISE_DESC_TILE
}

hipError_t launch_aead_records(bool decrypt, const uint8_t *keys,
                               uint32_t nkeys, const noise_gpu_record *recs,
                               uint64_t nrec, const uint8_t *in, uint8_t *out,
                               const uint8_t *ad, uint8_t *status,
                               hipStream_t stream) {
  if (nrec == 0) return hipSuccess;
  const dim3 bg(kGenBlock);
  const uint64_t gblocks = (nrec + kGenBlock - 1) / kGenBlock;
  if (nrec < kClassifyMin) {
    if (decrypt)
      hipLaunchKernelGGL((k_aead_records<true>), dim3((unsigned)gblocks), bg, 0, stream, keys, nkeys, recs, nrec, nullptr, nullptr, in, out, ad, status);
    else
      hipLaunchKernelGGL((k_aead_records<false>), dim3((unsigned)gblocks), bg, 0, stream, keys, nkeys, recs, nrec, nullptr, nullptr, in, out, ad, status);
    return hipGetLastError();
  }
  if (nrec > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit indices

  void *mem = nullptr;
  hipError_t e = scratch_get(&mem, sizeof(RecScratch) + 4 * nrec, stream);
  if (e != hipSuccess) return e;
  RecScratch *sc = static_cast<RecScratch *>(mem);
  uint32_t *idx = reinterpret_cast<uint32_t *>(sc + 1);
  e = hipMemsetAsync(sc, 0, sizeof(RecScratch), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_class_count, dim3((unsigned)gblocks), bg, 0, stream, recs, nrec, nkeys, in, out, sc);
  hipLaunchKernelGGL(k_class_scatter, dim3((unsigned)gblocks), bg, 0, stream, recs, nrec, nkeys, in, out, sc, idx);

  TileArgs ta{};
  ta.in = in;
  ta.out = out;
  ta.status = status;
  ta.keys = keys;
  ta.nkeys = nkeys;
  ta.recs = recs;
  ta.idx = idx;
  ta.counts = sc->counts;
  if (decrypt) launch_desc_tiles<true>(ta, nrec, stream);
  else launch_desc_tiles<false>(ta, nrec, stream);

  const uint64_t wblocks = (nrec + kWaveBatch - 1) / kWaveBatch;
  const dim3 gw((unsigned)(wblocks < NOISE_GRID_CAP ? wblocks : NOISE_GRID_CAP)), bw(64);
  if (decrypt)
    hipLaunchKernelGGL((k_aead_wave<true>), gw, bw, 0, stream, keys, nkeys, recs, idx, sc->counts, kClsWave, &sc->wave_cursor, in, out, status);
  else
    hipLaunchKernelGGL((k_aead_wave<false>), gw, bw, 0, stream, keys, nkeys, recs, idx, sc->counts, kClsWave, &sc->wave_cursor, in, out, status);

  const dim3 gg((unsigned)(gblocks < 2 * NOISE_GRID_CAP ? gblocks : 2 * NOISE_GRID_CAP));
  if (decrypt)
    hipLaunchKernelGGL((k_aead_records<true>), gg, bg, 0, stream, keys, nkeys, recs, nrec, idx, sc->counts, in, out, ad, status);
  else
    hipLaunchKernelGGL((k_aead_records<false>), gg, bg, 0, stream, keys, nkeys, recs, nrec, idx, sc->counts, in, out, ad, status);
  return hipGetLastError();
}

}  // namespace noise_amd
