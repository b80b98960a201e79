// records_kernels.hip -- descriptor batches (noise_gpu_{en,de}crypt_records):
// many sessions, mixed sizes (BASELINE config 4, the wavefront load-balance
// study).
//
// A batch of arbitrary records is load-balanced entirely on the device,
// stream-ordered (no host round trip):
//   1. classify (k_cls_count -> k_cls_scan -> k_cls_scatter): a counting
//      sort of descriptor indices by class with per-wave partial counts and
//      one scan -- no contended atomics;
//   2. one launch per class, each reading its slice and count from device
//      memory:
//        - tile classes: 16-byte aligned, AD-free records of any length up
//          to 2 KiB and of exactly 4, 8 and 16 KiB, by the smallest capacity
//          (64 .. 16384 B) that holds them -> the LDS-staged masked tile kernel (mtile_kernel.hpp,
//          kMTDesc), one launch per capacity for its exact-size and ragged
//          records;
//        - long records: 16-byte aligned, AD-free, 2 KiB < len <= 65535
//          except exactly 4, 8, 16 KiB (see record_class) -> cut into 1 KiB
//          segments + a tail (masked 1 KiB tile units).  k_seg_prep
//          derives each record's one-time key and r powers, ONE tile-kernel
//          launch (kTileSeg) encrypts every full segment of every long
//          record -- uniform 1 KiB work units, whatever the size mix -- and
//          k_seg_finalize_w combines the segments' Poly1305 partial sums with
//          the tail's, the length block and the tag.  Decrypt verifies first:
//          a Poly1305-only pass over the ciphertext (kTileSegPoly, kMTTailPoly),
//          the finalize checks every tag, and only then the keystream pass
//          (kTileSegXor, kMTTailXor) writes the plaintext of the records that
//          verified -- no byte of a failed record's plaintext is ever stored;
//        - generic: everything else (AD, unaligned, bad key index, > 65535
//          bytes, and long records beyond the segment scratch capacity)
//          -> one lane per record (chachapoly_device.hpp).
// Small batches (< kClassifyMin records) skip all this and run the generic
// kernel directly (latency of single records from CipherState).
// Scratch is a grow-only device buffer cached per (device, stream).
#include <mutex>
#include <vector>

#include "chachapoly_device.hpp"
#include "launchers.hpp"
#include "mtile_kernel.hpp"
#include "noise_amd/dev_mem.hpp"
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kGenBlock = 256;
constexpr int kNumTileCls = 10;           // exactly 64 128 192 256 512 1024 2048 4096 8192 16384
constexpr int kMCls0 = kNumTileCls;       // the masked (ragged) classes: any other length up to
constexpr int kNumMCls = 10;              //   the same ten capacities (mtile_kernel.hpp)
static_assert(kNumMCls == kNumTileCls, "one ragged class per exact tile class");
// idx order: exact class c, then the ragged class of the same capacity (one
// masked-kernel launch takes both: launch_classes), then long and generic
__host__ __device__ constexpr int cls_order(int k) {
  return k < 2 * kNumTileCls ? ((k & 1) ? kMCls0 + k / 2 : k / 2) : k;
}
constexpr int kClsLong = kMCls0 + kNumMCls;  // segmented long records (> 16 KiB)
constexpr int kClsGeneric = kClsLong + 1;
constexpr int kNumCls = kClsLong + 2;
constexpr int kColSegs = kNumCls;         // classifier column: full segments
constexpr int kColTails = kNumCls + 1;    // classifier column: long records with a tail
constexpr int kColFin0 = kNumCls + 2;     // classifier columns: long records by
constexpr int kFinBuckets = 6;            // floor(log2(full segments)), 1..63 -> 0..5
constexpr int kCols = kNumCls + 2 + kFinBuckets;
// Decrypt pipelines the long records in kSegChunks chunks (launch_classes):
// the Poly1305 pass of chunk c + 1 (HBM-bound) runs beside the keystream pass
// of chunk c (VALU-bound).  Chunk boundaries fall on record starts, near
// (1 + (c - 1) W) nseg / (1 + (kSegChunks - 1) W) segments (chunk 0 1/W of
// the others, W = kChunkW).
#ifndef NOISE_SEG_CHUNKS
#define NOISE_SEG_CHUNKS 4
#endif
constexpr int kSegChunks = NOISE_SEG_CHUNKS;
#ifndef NOISE_CHUNK_W
#define NOISE_CHUNK_W 4
#endif
constexpr unsigned long long kChunkW = NOISE_CHUNK_W;  // chunk c >= 1 : chunk 0
#ifndef NOISE_CHUNK_MIN  // overridable for the CPU emulation build
#define NOISE_CHUNK_MIN 65536
#endif
constexpr uint64_t kChunkMinRecords = NOISE_CHUNK_MIN;  // smaller batches: one chunk
constexpr int kHdrWords = kSegChunks <= 4 ? 128 : 256;    // scratch header: 1 KiB (2 KiB)
// finalize lanes per long record
#ifndef NOISE_FIN_W
#define NOISE_FIN_W 4
#endif
// The XOR pass's span per lane: 128 B halves its LDS tile (8 segments, 8 KiB)
// so that, at its ~120 VGPRs, four waves fit per SIMD (256 B: 16.6 KiB per
// wave, 2.25 waves per SIMD by LDS).  Same box, config 4 (round 4):
// 3.54-3.61 ms per decrypt against 3.83-3.90 at 256 B.
#ifndef NOISE_XOR_SPAN
#define NOISE_XOR_SPAN 128
#endif
// The Poly1305 pass's span per lane: 256 B, as the encrypt segment kernel
// (one recombination product per lane with the SegRec's powers; 128-B spans
// would need r^8 .. r^56).  Round 5, per-kernel PMC: 53 M VALU per chunk
// against 79 M for 128-B spans with a three-product recombination.
#ifndef NOISE_POLY_SPAN
#define NOISE_POLY_SPAN 256
#endif
// classifier geometry: waves (a multiple of 64) and the least records per wave
#ifndef NOISE_CLS_WAVES
#define NOISE_CLS_WAVES 4096  // round 5: 2048 waves of >= 512 ran 0.5 % slower per call
#endif
#ifndef NOISE_CLS_MIN_CHUNK
#define NOISE_CLS_MIN_CHUNK 256
#endif
constexpr uint32_t kClsWaves = NOISE_CLS_WAVES;
constexpr uint64_t kClsMinChunk = NOISE_CLS_MIN_CHUNK;
static_assert(kClsWaves % 64 == 0 && kClsMinChunk % 64 == 0, "classifier geometry");
#ifndef NOISE_CLASSIFY_MIN  // overridable for the CPU emulation build
#define NOISE_CLASSIFY_MIN 2048
#endif
constexpr uint64_t kClassifyMin = NOISE_CLASSIFY_MIN;
constexpr uint64_t kClassifyAvgLen = 2048;  // below kClassifyMin: classify when records average this
constexpr uint32_t kLongMax = 65535;      // the Noise message bound
#ifndef NOISE_SEG_CAP  // overridable for the CPU emulation build (overflow path)
#define NOISE_SEG_CAP (1ull << 24)
#endif
constexpr uint64_t kSegCapMax = NOISE_SEG_CAP;  // 16 Mi segments = 16 GiB per call
// Grid cap of the per-class launches, whose sizes are known only on the
// device (capped grids stride over their work).  8192 single-wave workgroups
// = 4x what the LDS budget keeps resident (8 per CU): the dispatcher refills
// CUs as workgroups finish, which balanced config 4 best (2048: -6 %, 16384
// and uncapped: -3 %, MI355X).  Overridable for the CPU emulation build.
#ifndef NOISE_GRID_CAP
#define NOISE_GRID_CAP 8192u
#endif

// an all-zero key row is "no key" (Noise HasKey() false, e.g. the rows
// noise_gpu_hs_split leaves for failed handshakes): never used to encrypt
__device__ __forceinline__ bool key_row_zero(const uint8_t *keys, uint32_t ki) {
  const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 32ull * ki);
  const uint4 a = kp[0], b = kp[1];
  return (a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) == 0u;
}

// (NOISE_SEG_LO, NOISE_SEG_MID_HI] (not an exact tile size): segments
// instead of the masked tile of the next capacity
#ifndef NOISE_SEG_LO
#define NOISE_SEG_LO 2048
#endif
#ifndef NOISE_SEG_MID_HI
#define NOISE_SEG_MID_HI 16383
#endif

// records the tile / segment kernels cannot take go to the generic class,
// which also reports bad key rows (index out of range or all zero)
__device__ __forceinline__ int record_class(const noise_gpu_record &d, const uint8_t *keys,
                                            uint32_t nkeys, const uint8_t *in,
                                            const uint8_t *out) {
  if (d.key_idx >= nkeys || d.ad_len != 0 || d.len == 0) return kClsGeneric;
  if (key_row_zero(keys, d.key_idx)) return kClsGeneric;
  if (((reinterpret_cast<uintptr_t>(in + d.in_off) |
        reinterpret_cast<uintptr_t>(out + d.out_off)) & 15u) != 0)
    return kClsGeneric;
  switch (d.len) {
    case 64: return 0;
    case 128: return 1;
    case 192: return 2;
    case 256: return 3;
    case 512: return 4;
    case 1024: return 5;  // exactly 1 KiB: one tile-kernel pass beats prep + segment + finalize
    // whole-record tiles up to 16 KiB (one 16 KiB LDS tile per record at
    // 16 KiB): the tag is computed and checked in the wave that holds the
    // record, so decrypt reads it once -- the segment path's verify-first
    // decrypt reads a long record's ciphertext twice (§4.3 of DESIGN.md)
    case 2048: return 6;
    case 4096: return 7;
    case 8192: return 8;
    case 16384: return 9;
    default: break;
  }
  // every other length up to 16 KiB: the masked tile class of the smallest
  // capacity that holds it -- the record still sits whole in one wave's
  // tile, so decrypt checks its tag there and reads the ciphertext once
  // Above 2 KiB (but the exact 4, 8, 16 KiB tiles) the segment path (1 KiB
  // segments + a masked tail unit) beats the masked tile of the next
  // capacity: single-length batches of 3000 / 5000 / 9000 / 16000 B at
  // 1131 / 1205 / 1223 / 1219 GiB/s against 983 / 813 / 693 / 1148, config 4
  // within its noise (profiles/round6/ab/seg_threshold.md)
  if (d.len <= 16384u && !(d.len > (uint32_t)NOISE_SEG_LO && d.len <= (uint32_t)NOISE_SEG_MID_HI)) {
    const uint32_t n = d.len;
    const int c = n <= 64u ? 0 : n <= 128u ? 1 : n <= 192u ? 2 : n <= 256u ? 3 : n <= 512u ? 4
                : n <= 1024u ? 5 : n <= 2048u ? 6 : n <= 4096u ? 7 : n <= 8192u ? 8 : 9;
    return kMCls0 + c;
  }
  return d.len <= kLongMax ? kClsLong : kClsGeneric;
}

// device header of the scratch buffer
struct RecHdr {
  unsigned long long counts[kCols];    // records per class; [kColSegs] = segments,
                                       // [kColTails] = tails
  unsigned long long cls_base[kCols];  // start of each class in idx
  unsigned long long nlong;            // long records handled as segments
  unsigned long long nseg;             // their full segments
  unsigned long long spare0;
  // chunk c = long records [qsplit[c], qsplit[c + 1]) = segments [ssplit[c],
  // ssplit[c + 1]) (k_cls_scatter; clamped to nlong / nseg where used)
  // and tails [tsplit[c], tsplit[c + 1]) (clamped to the tail count)
  unsigned long long qsplit[kSegChunks + 1], ssplit[kSegChunks + 1], tsplit[kSegChunks + 1];
  unsigned long long pad[kHdrWords - 3 - 2 * kCols - 3 * (kSegChunks + 1)];
};
static_assert(sizeof(RecHdr) == 8 * kHdrWords, "scratch header layout");

// finalize-order bucket of a long record with nf >= 1 full segments
__device__ __forceinline__ int fin_bucket(uint32_t nf) {
  const int b = 31 - __builtin_clz(nf | 1u);
  return b < kFinBuckets - 1 ? b : kFinBuckets - 1;
}

// wave-wide inclusive prefix sum (all 64 lanes participate)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl((int)v, (int)(lane >= (uint32_t)d ? lane - d : lane));
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_incl_scan64(unsigned long long v,
                                                               uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int src = (int)(lane >= (uint32_t)d ? lane - d : lane);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    if (lane >= (uint32_t)d) v += ((unsigned long long)hi << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v += (uint32_t)__shfl_xor((int)v, d);
  return v;
}

// ---- 1. classification ------------------------------------------------------
// Wave w owns records [w*chunk, (w+1)*chunk).  Per-wave partial counts go
// to part[w][col]; one wave scans them; the scatter pass writes the sorted
// index array (class order, record order within a class) and, for long
// records, their SegRec header fields and the segment list.
__global__ __launch_bounds__(64) void k_cls_count(
    const noise_gpu_record *__restrict__ recs, uint64_t nrec, uint32_t chunk,
    const uint8_t *keys, uint32_t nkeys, const uint8_t *in, const uint8_t *out, uint32_t *part) {
  const uint32_t lane = threadIdx.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
  const uint64_t e0 = b0 + chunk < nrec ? b0 + chunk : nrec;
  uint32_t cnt[kNumCls] = {0}, fin[kFinBuckets] = {0}, nseg = 0, ntail = 0;
#pragma unroll 1
  for (uint64_t i0 = b0; i0 < e0; i0 += 64) {
    const uint64_t i = i0 + lane;
    int cls = -1;
    uint32_t nf = 0;
    bool tail = false;
    if (i < e0) {
      const noise_gpu_record d = recs[i];
      cls = record_class(d, keys, nkeys, in, out);
      nf = cls == kClsLong ? d.len >> 10 : 0u;
      tail = cls == kClsLong && (d.len & 1023u) != 0;
    }
#pragma unroll
    for (int c = 0; c < kNumCls; ++c) cnt[c] += (uint32_t)__builtin_popcountll(__ballot(cls == c));
    nseg += wave_sum(nf);
    ntail += (uint32_t)__builtin_popcountll(__ballot(tail));
    const int fb = cls == kClsLong ? fin_bucket(nf) : -1;
#pragma unroll
    for (int b = 0; b < kFinBuckets; ++b) fin[b] += (uint32_t)__builtin_popcountll(__ballot(fb == b));
  }
  if (lane < (uint32_t)kCols) {
    uint32_t v = lane == (uint32_t)kColSegs ? nseg : ntail;
#pragma unroll
    for (int c = 0; c < kNumCls; ++c) v = lane == (uint32_t)c ? cnt[c] : v;
#pragma unroll
    for (int b = 0; b < kFinBuckets; ++b) v = lane == (uint32_t)(kColFin0 + b) ? fin[b] : v;
    part[(uint64_t)blockIdx.x * kCols + lane] = v;
  }
}

// one workgroup per column.  Lane l owns the contiguous waves
// [l*per, (l+1)*per): all its loads go out together (one memory round trip
// instead of one per 64 waves), then a local prefix, a wave scan of the lane
// totals, and the bases are written back.
__global__ __launch_bounds__(64) void k_cls_scan(const uint32_t *part, uint32_t nw,
                                                 unsigned long long *wbase,
                                                 RecHdr *hdr, uint64_t segcap) {
  const uint32_t lane = threadIdx.x, c = blockIdx.x;
  constexpr uint32_t kPer = kClsWaves / 64;  // nw <= kClsWaves (the classifier's geometry)
  const uint32_t w0 = lane * kPer;
  uint32_t v[kPer];
  unsigned long long tot = 0;  // 32 waves' segment counts can pass 2^32
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    v[i] = w0 + i < nw ? part[(uint64_t)(w0 + i) * kCols + c] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) tot += v[i];
  const unsigned long long inc = wave_incl_scan64(tot, lane);
  unsigned long long run = inc - tot;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    if (w0 + i < nw) wbase[(uint64_t)(w0 + i) * kCols + c] = run;
    run += v[i];
  }
  if (lane == 63) {
    hdr->counts[c] = run;
    // lowered by k_cls_scatter if the segment scratch overflows
    if (c == (uint32_t)kClsLong) {
      hdr->nlong = run;
      hdr->spare0 = 0;
    }
    if (c == (uint32_t)kColSegs) {
      hdr->nseg = run < segcap ? run : segcap;
      // chunk c >= 1 starts at the record holding segment c * nseg / chunks
      // (k_cls_scatter writes it; none holds it when there are no segments)
      for (int k = 0; k <= kSegChunks; ++k) {
        hdr->qsplit[k] = k == 0 ? 0ull : ~0ull;
        hdr->ssplit[k] = k == 0 ? 0ull : ~0ull;
        hdr->tsplit[k] = k == 0 ? 0ull : ~0ull;
      }
    }
  }
}

__global__ __launch_bounds__(64) void k_cls_scatter(
    const noise_gpu_record *__restrict__ recs, uint64_t nrec, uint32_t chunk,
    const uint8_t *keys, uint32_t nkeys, const uint8_t *in, const uint8_t *out,
    const unsigned long long *wbase, RecHdr *hdr, uint32_t *idx, SegRec *rt,
    SegEntry *segs, uint32_t *tails, uint32_t *fin, uint64_t segcap) {
  const uint32_t lane = threadIdx.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
  const uint64_t e0 = b0 + chunk < nrec ? b0 + chunk : nrec;
  unsigned long long run[kCols];
#pragma unroll
  for (int c = 0; c < kCols; ++c) run[c] = wbase[(uint64_t)blockIdx.x * kCols + c];
  unsigned long long cbase[kNumCls];
  {
    unsigned long long b = 0;
#pragma unroll
    for (int k = 0; k < kNumCls; ++k) {
      const int c = cls_order(k);
      cbase[c] = b;
      b += hdr->counts[c];
    }
  }
  unsigned long long fbase[kFinBuckets];
  {
    unsigned long long b = 0;
#pragma unroll
    for (int c = 0; c < kFinBuckets; ++c) {
      fbase[c] = b;
      b += hdr->counts[kColFin0 + c];
    }
  }
  if (blockIdx.x == 0 && lane < (uint32_t)kNumCls) {
    unsigned long long b = cbase[0];
#pragma unroll
    for (int c = 0; c < kNumCls; ++c) b = lane == (uint32_t)c ? cbase[c] : b;
    hdr->cls_base[lane] = b;
  }
  bool overflow = false;
  unsigned long long ov_q = ~0ull, ov_seg = ~0ull;
#pragma unroll 1
  for (uint64_t i0 = b0; i0 < e0; i0 += 64) {
    const uint64_t i = i0 + lane;
    int cls = -1;
    noise_gpu_record d{};
    if (i < e0) {
      d = recs[i];
      cls = record_class(d, keys, nkeys, in, out);
    }
    const uint32_t nf = cls == kClsLong ? d.len >> 10 : 0u;
    const bool tail = cls == kClsLong && (d.len & 1023u) != 0;
    unsigned long long q = 0;
#pragma unroll
    for (int c = 0; c < kNumCls; ++c) {
      const uint64_t m = __ballot(cls == c);
      if (cls == c) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        q = run[c] + rank;
        idx[cbase[c] + q] = (uint32_t)i;
      }
      run[c] += (unsigned long long)__builtin_popcountll(m);
    }
    {  // long records in finalize order: by segment-count bucket
      const int fb = cls == kClsLong ? fin_bucket(nf) : -1;
#pragma unroll
      for (int b = 0; b < kFinBuckets; ++b) {
        const uint64_t m = __ballot(fb == b);
        if (fb == b)
          fin[fbase[b] + run[kColFin0 + b] +
              __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              (uint32_t)q;
        run[kColFin0 + b] += (unsigned long long)__builtin_popcountll(m);
      }
    }
    unsigned long long tpos;  // tails of the records before this lane's
    {  // long records with a tail: the tail list (record order)
      const uint64_t m = __ballot(tail);
      tpos = run[kColTails] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (tail) tails[tpos] = (uint32_t)q;
      run[kColTails] += (unsigned long long)__builtin_popcountll(m);
    }
    // long records: header fields of their SegRec, first segment index
    const uint32_t inc = wave_incl_scan(nf, lane);
    const uint32_t total = (uint32_t)__shfl((int)inc, 63);
    const uint32_t rel0 = inc - nf;
    if (cls == kClsLong) {
      const unsigned long long seg0 = run[kColSegs] + rel0;
      SegRec &R = rt[q];
      R.in_off = d.in_off;
      R.out_off = d.out_off;
      R.nonce = d.nonce;
      R.seg0 = seg0;
      R.key_idx = d.key_idx;
      R.di = (uint32_t)i;
      R.len = d.len;
      R.nfull = nf;
      if (seg0 + nf > segcap) {  // beyond the scratch: this and later long records go generic
        overflow = true;
        ov_q = q < ov_q ? q : ov_q;
        ov_seg = seg0 < ov_seg ? seg0 : ov_seg;
      }
      const unsigned long long total = hdr->counts[kColSegs];
#pragma unroll
      for (int k = 1; k < kSegChunks; ++k) {  // the record holding a chunk's first segment
        // chunk 0 smaller than the others (1 : W : W : ...): the first tag
        // check, and so the keystream pass, can start sooner
        const unsigned long long b = total * (1ull + (k - 1ull) * kChunkW) / (1ull + (kSegChunks - 1ull) * kChunkW);
        if (seg0 <= b && b < seg0 + nf) {
          hdr->qsplit[k] = q;
          hdr->ssplit[k] = seg0;
          hdr->tsplit[k] = tpos;
        }
      }
    }
    // segment list entries (q, s), written cooperatively: entry k of this
    // group belongs to the first lane whose inclusive count exceeds k
#pragma unroll 1
    for (uint32_t k0 = 0; k0 < total; k0 += 64) {
      const uint32_t k = k0 + lane;
      uint32_t lo = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t probe = (uint32_t)__shfl((int)inc, (int)(lo + step - 1));
        if (probe <= k) lo += step;
      }
      const uint32_t oq = (uint32_t)__shfl((int)(uint32_t)q, (int)lo);
      const uint32_t orel = (uint32_t)__shfl((int)rel0, (int)lo);
      const unsigned long long pos = run[kColSegs] + k;
      if (k < total && pos < segcap) segs[pos] = SegEntry{oq, k - orel};
    }
    run[kColSegs] += total;
  }
  if (overflow) {  // rare: only when the long records exceed kSegCapMax segments
    atomicMin(&hdr->nlong, ov_q);
    atomicMin(&hdr->nseg, ov_seg);
  }
}

// ---- 2. long records --------------------------------------------------------
// k_seg_prep: lane per long record -> ChaCha block 0 (one-time key r, s),
// r^16, r^32, r^48 (the segment passes' per-lane recombination) and r^64
// (the finalize kernel's Horner step over segments).
__global__ __launch_bounds__(64) void k_seg_prep(const uint8_t *__restrict__ keys,
                                                 SegRec *rt, const RecHdr *hdr) {
  const uint64_t n = hdr->nlong;
#pragma unroll 1
  for (uint64_t q = (uint64_t)blockIdx.x * 64 + threadIdx.x; q < n;
       q += (uint64_t)gridDim.x * 64) {
    SegRec &R = rt[q];
    const u32x4 *kp = reinterpret_cast<const u32x4 *>(keys + 32ull * R.key_idx);
    const u32x4 ka = kp[0], kb = kp[1];
    const uint32_t k[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) R.k[i] = k[i];
    uint32_t otk[16];
    chacha20_block(k, 0u, (uint32_t)R.nonce, (uint32_t)(R.nonce >> 32), otk);
    const uint32_t r0 = otk[0] & 0x0fffffffu, r1 = otk[1] & 0x0ffffffcu,
                   r2 = otk[2] & 0x0ffffffcu, r3 = otk[3] & 0x0ffffffcu;
    R.r[0] = r0; R.r[1] = r1; R.r[2] = r2; R.r[3] = r3;
    R.s[0] = otk[4]; R.s[1] = otk[5]; R.s[2] = otk[6]; R.s[3] = otk[7];
    // squaring chain r^(2^b); r^(tail blocks) = product over the bits of
    // the tail's Poly1305 block count (1..64)
    const uint32_t nbt = ((R.len & 1023u) + 15u) >> 4;
    F26 x = to26(r0, r1, r2, r3, 0u), rt_pow, xb[4];
    rt_pow.a[0] = 1u;
    rt_pow.a[1] = rt_pow.a[2] = rt_pow.a[3] = rt_pow.a[4] = 0u;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xb[b] = x;  // r^(2^b)
      if ((nbt >> b) & 1u) rt_pow = mul26(rt_pow, x);
      x = mul26(x, x);
    }
    {  // r^(16 - t) for the tail's masked tile unit (t = 4 ceil(tail / 64) - nbt)
      const uint32_t t = 4u * (((R.len & 1023u) + 63u) >> 6) - nbt;
      F26 y = t ? mul26(xb[3], xb[2]) : x;       // r^12 (r^16 when t = 0)
      if (t == 1u || t == 2u) y = mul26(y, xb[1]);
      if (t == 1u || t == 3u) y = mul26(y, xb[0]);
#pragma unroll
      for (int i = 0; i < 5; ++i) R.r16t[i] = y.a[i];
    }
    // x = r^16
    if ((nbt >> 4) & 1u) rt_pow = mul26(rt_pow, x);
    const F26 x32 = mul26(x, x), x64 = mul26(x32, x32);
    if ((nbt >> 5) & 1u) rt_pow = mul26(rt_pow, x32);
    if ((nbt >> 6) & 1u) rt_pow = mul26(rt_pow, x64);  // a 1009..1023-byte tail: 64 blocks
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      R.r64[i] = x64.a[i];
      R.rtail[i] = rt_pow.a[i];
    }
    const F26 pw[3] = {x, x32, mul26(x32, x)};
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      *reinterpret_cast<u32x4 *>(R.pwlo[m]) = u32x4{pw[m].a[0], pw[m].a[1], pw[m].a[2], pw[m].a[3]};
      R.pwhi[m] = pw[m].a[4];
    }
  }
}

// k_seg_finalize_w: W lanes per long record (a group; a wave finalizes 64 / W
// records of similar segment count per pass -- the classifier's segment-count
// buckets -- so a 63-segment record is not one lane's chain of 63 dependent
// products and load round trips).  h = the Horner sum of the segments'
// partial sums in R = r^64, then h r^(tail blocks) + P_tail, the length block
// and the tag: encrypt stores it; decrypt compares it, writes the record's
// status and its SegRec.ok, which the plaintext passes (kTileSegXor,
// kTailXor) read.  Group lane i takes segments i, i + W, ... (loaded
// together) and runs Horner in R^W:
//   acc_i = sum_k P_{i+Wk} R^(W(K_i-1-k)),   K_i = ceil((nf - i) / W)
// then h = sum_i acc_i R^(e_i) with e_i = nf-1 - (i + W(K_i-1)) in [0, W)
// (log2 W selected products by R, R^2, ...) and a log2 W-level xor butterfly
// over the group.  Group lane 0 then appends the tail and writes / checks the
// tag exactly as k_seg_finalize does.  Every lane repeats the log2 W
// squarings, so W trades chain length for redundant products: W = 4 keeps
// the whole call cheaper than one lane per record (W = 8 is VALU-bound on
// the squarings).
template <bool DECRYPT, int W>
__global__ __launch_bounds__(64) void k_seg_finalize_w(
    const uint32_t *__restrict__ fin, SegRec *__restrict__ rt,
    const SegPartial *__restrict__ partial, const uint32_t *__restrict__ partial_hi,
    RecHdr *hdr, const uint8_t *in, uint8_t *out, uint8_t *status, int chunk) {
  static_assert(W == 2 || W == 4 || W == 8, "lanes per record");
  constexpr int LOGW = W == 2 ? 1 : (W == 4 ? 2 : 3);
  constexpr uint32_t KMAX = (63u + W - 1u) / W;  // segments per lane (nf <= 63)
  const uint64_t nlong = hdr->nlong;
  // chunk < 0: every long record, in the classifier's bucket order (fin);
  // chunk c: the records [qsplit[c], qsplit[c + 1]) in record order
  uint64_t n = hdr->counts[kClsLong], q0 = 0;
  if (chunk >= 0) {
    const uint64_t lo = hdr->qsplit[chunk], hi = hdr->qsplit[chunk + 1];
    q0 = lo < nlong ? lo : nlong;
    n = (hi < nlong ? hi : nlong) - q0;
  }
  const uint32_t i = threadIdx.x & (W - 1u);
#pragma unroll 1
  for (uint64_t base = (uint64_t)blockIdx.x * (64 / W); base < n;
       base += (uint64_t)gridDim.x * (64 / W)) {
    // every lane stays in the loop body (the butterfly reads all group
    // lanes); a group without a record works on zeros and stores nothing
    const uint64_t t = base + (threadIdx.x / W);
    uint32_t q = t < n ? (chunk >= 0 ? (uint32_t)(q0 + t) : fin[t]) : 0xffffffffu;
    const bool ok = q < nlong;
    if (!ok) q = 0;
    uint32_t nf = 0;
    uint64_t seg0 = 0;
    F26 pw[LOGW + 1];  // R^(2^b), b = 0 .. LOGW
#pragma unroll
    for (int k = 0; k < 5; ++k) pw[0].a[k] = k == 0 ? 1u : 0u;
    if (ok) {
      const SegRec &R = rt[q];
      nf = R.nfull;
      seg0 = R.seg0;
#pragma unroll
      for (int k = 0; k < 5; ++k) pw[0].a[k] = R.r64[k];
    }
    // this lane's segments, all loads in flight together
    const uint32_t K = nf > i ? (nf - i + W - 1u) / W : 0u;
    uint4 lo[KMAX];
    uint32_t hi[KMAX];
#pragma unroll
    for (uint32_t k = 0; k < KMAX; ++k) {
      lo[k] = make_uint4(0u, 0u, 0u, 0u);
      hi[k] = 0u;
      if (k < K) {
        const SegPartial &P = partial[seg0 + i + W * k];
        lo[k] = make_uint4(P.h[0], P.h[1], P.h[2], P.h[3]);
        hi[k] = partial_hi[seg0 + i + W * k];
      }
    }
#pragma unroll
    for (int b = 1; b <= LOGW; ++b) pw[b] = mul26(pw[b - 1], pw[b - 1]);
    F26 acc = to26(lo[0].x, lo[0].y, lo[0].z, lo[0].w, hi[0]);  // zeros when K == 0
#pragma unroll
    for (uint32_t k = 1; k < KMAX; ++k) {
      if (k < K) {
        acc = mul26(acc, pw[LOGW]);
        const F26 v = to26(lo[k].x, lo[k].y, lo[k].z, lo[k].w, hi[k]);
#pragma unroll
        for (int m = 0; m < 5; ++m) acc.a[m] += v.a[m];
        carry26(acc);
      }
    }
    // * R^(e_i): the lane's last segment is followed by e_i more
    const uint32_t e = K ? nf - 1u - i - W * (K - 1u) : 0u;
#pragma unroll
    for (int b = 0; b < LOGW; ++b) {
      F26 f;
      const bool use = (e >> b) & 1u;
#pragma unroll
      for (int m = 0; m < 5; ++m) f.a[m] = use ? pw[b].a[m] : (m == 0 ? 1u : 0u);
      acc = mul26(acc, f);
    }
    // limbs < 2^26 + 2^9 after mul26: the group's sum fits in 32 bits
#pragma unroll
    for (int b = 1; b < W; b <<= 1) {
#pragma unroll
      for (int m = 0; m < 5; ++m) acc.a[m] += (uint32_t)__shfl_xor((int)acc.a[m], b);
    }
    if (i != 0 || !ok) continue;
    SegRec &R = rt[q];
    const uint32_t len = R.len;
    if (len & 1023u) {
      carry26(acc);
      F26 rtp;
#pragma unroll
      for (int m = 0; m < 5; ++m) rtp.a[m] = R.rtail[m];
      acc = mul26(acc, rtp);
      const F26 v = to26(R.ptail[0], R.ptail[1], R.ptail[2], R.ptail[3], R.ptail[4]);
#pragma unroll
      for (int m = 0; m < 5; ++m) acc.a[m] += v.a[m];
    }
    carry26(acc);
    carry26(acc);
    Poly1305 p;
    from26(acc, p.h0, p.h1, p.h2, p.h3, p.h4);
    p.r0 = R.r[0]; p.r1 = R.r[1]; p.r2 = R.r[2]; p.r3 = R.r[3];
    p.rr0 = (p.r0 >> 2) * 5u;
    p.rr1 = p.r1 + (p.r1 >> 2);
    p.rr2 = p.r2 + (p.r2 >> 2);
    p.rr3 = p.r3 + (p.r3 >> 2);
    p.r0lo = p.r0 & 3u;
    p.s0 = R.s[0]; p.s1 = R.s[1]; p.s2 = R.s[2]; p.s3 = R.s[3];
    poly_block(p, 0u, 0u, len, 0u);  // LE64(ad_len = 0) || LE64(len)
    uint32_t tag[4];
    poly_final(p, tag);
    if (!DECRYPT) {
      uint8_t *tp = out + R.out_off + len;
      if ((len & 15u) == 0) store16<true>(tp, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
      else store16<false>(tp, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
    } else {
      const uint8_t *tp = in + R.in_off + len;
      const uint4 want = (len & 15u) == 0 ? load16<true>(tp, 16) : load16<false>(tp, 16);
      const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) |
                            (want.w ^ tag[3]);
      status[R.di] = diff == 0u ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
      R.ok = diff == 0u ? 1u : 0u;  // the plaintext passes write only verified records
    }
  }
}

// ---- generic: one lane per record ------------------------------------------
// idx == nullptr: record i directly (small batches).  Otherwise the generic
// class, followed by the long records the segment scratch could not take.
template <bool DECRYPT>
__global__ __launch_bounds__(kGenBlock) void k_aead_records(
    const uint8_t *__restrict__ keys, uint32_t nkeys,
    const noise_gpu_record *__restrict__ recs, uint64_t nrec,
    const uint32_t *__restrict__ idx, const RecHdr *hdr,
    const uint8_t *in, uint8_t *out, const uint8_t *ad, uint8_t *status) {
  uint64_t base = 0, n = nrec, base2 = 0, n2 = 0;
  if (idx) {
    base = hdr->cls_base[kClsGeneric];
    n = hdr->counts[kClsGeneric];
    base2 = hdr->cls_base[kClsLong] + hdr->nlong;
    n2 = hdr->counts[kClsLong] - hdr->nlong;
  }
#pragma unroll 1
  for (uint64_t i = (uint64_t)blockIdx.x * kGenBlock + threadIdx.x; i < n + n2;
       i += (uint64_t)gridDim.x * kGenBlock) {
    const uint64_t di = idx ? idx[i < n ? base + i : base2 + (i - n)] : i;
    const noise_gpu_record r = recs[di];
    if (r.key_idx >= nkeys) {  // never index outside the key table
      if (DECRYPT) status[di] = NOISE_GPU_REC_BAD_KEY;
      continue;
    }
    const uint4 *kp = reinterpret_cast<const uint4 *>(keys + 32ull * r.key_idx);
    const uint4 ka = kp[0], kb = kp[1];
    const uint32_t k[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
    if ((ka.x | ka.y | ka.z | ka.w | kb.x | kb.y | kb.z | kb.w) == 0u) {  // no key
      if (DECRYPT) status[di] = NOISE_GPU_REC_BAD_KEY;
      continue;
    }
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
// Calls on one stream are ordered, so they may share the buffer.  It only
// grows; the smaller one is wiped and freed stream-ordered (dev_mem.hpp), so
// it is released after the launches that still use it, and the grow waits for
// nothing else on the device (hipFree would wait for every stream, e.g. for a
// resident latency instance serving another thread).
struct ScratchEntry {
  int dev;
  hipStream_t stream;
  void *ptr;
  size_t size;
};
static std::mutex g_scratch_mu;
static std::vector<ScratchEntry> g_scratch;

static void scratch_find(int dev, hipStream_t stream, void **p, size_t *size) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (const ScratchEntry &en : g_scratch)
    if (en.dev == dev && en.stream == stream) {
      *p = en.ptr;
      *size = en.size;
      return;
    }
}

static hipError_t scratch_get(void **p, size_t bytes, hipStream_t stream) {
  using Entry = ScratchEntry;
  auto &mu = g_scratch_mu;
  auto &cache = g_scratch;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  for (Entry &en : cache) {
    if (en.dev != dev || en.stream != stream) continue;
    if (en.size < bytes) {
      if ((e = dev_wipe_free(en.ptr, en.size, stream)) != hipSuccess) return e;
      en.ptr = nullptr;
      en.size = 0;
      if ((e = dev_alloc(&en.ptr, bytes, stream)) != hipSuccess) return e;
      en.size = bytes;
    }
    *p = en.ptr;
    return hipSuccess;
  }
  void *ptr = nullptr;
  if ((e = dev_alloc(&ptr, bytes, stream)) != hipSuccess) return e;
  cache.push_back({dev, stream, ptr, bytes});
  *p = ptr;
  return hipSuccess;
}

hipError_t records_scratch_get(void **p, size_t bytes, hipStream_t stream) {
  return scratch_get(p, bytes, stream);
}

// Zero the scratch of (current device, stream): the long-record table holds
// key copies, one-time Poly1305 keys and partial sums between the kernels of
// a call.  Stream-ordered after the call's kernels.
hipError_t records_scratch_wipe(hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  void *ptr = nullptr;
  size_t size = 0;
  scratch_find(dev, stream, &ptr, &size);
  if (!ptr) return hipSuccess;
  return hipMemsetAsync(ptr, 0, size, stream);
}

// Release everything cached for (current device, stream): the scratch is
// zeroed and freed, the companion stream and its events destroyed.  Called
// before a stream the engine owns is destroyed (noise_gpu_ctx_destroy,
// per-thread staging teardown), so neither a dead stream's scratch nor its
// companion outlives it.  Synchronises `stream` first.
static hipError_t aux_release(int dev, hipStream_t stream);
hipError_t records_scratch_release(hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  void *ptr = nullptr;
  size_t size = 0;
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (size_t i = 0; i < g_scratch.size(); ++i)
      if (g_scratch[i].dev == dev && g_scratch[i].stream == stream) {
        ptr = g_scratch[i].ptr;
        size = g_scratch[i].size;
        g_scratch.erase(g_scratch.begin() + (std::ptrdiff_t)i);
        break;
      }
  }
  if (ptr) e = dev_wipe_free(ptr, size, stream);  // after the calls queued on `stream`
  const hipError_t e2 = hipStreamSynchronize(stream);
  if (e == hipSuccess) e = e2;
  const hipError_t e3 = aux_release(dev, stream);
  return e == hipSuccess ? e3 : e;
}

static inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
static inline unsigned capped(uint64_t want, uint64_t cap) {
  if (want == 0) want = 1;
  return (unsigned)(want < cap ? want : cap);
}

// Fork/join companion of a caller stream: a non-blocking stream and two
// events, cached per (device, stream) like the scratch.  The records DAG has
// two independent branches after the classifier (below); the short ones run
// on the companion stream while the segment kernel fills the GPU.
struct AuxStream {
  hipStream_t aux = nullptr;   // companion: small classes, generic, tails
  hipStream_t aux2 = nullptr;  // decrypt: per chunk, tag check + plaintext pass
  hipStream_t aux3 = nullptr;  // the whole-record classes of 2 .. 16 KiB
  // fork: classifier done; prep: k_seg_prep done; join: encrypt: the
  // companion branch done, decrypt: the tails' Poly1305 done; join2: the
  // companion done (decrypt); xdone: the last plaintext pass done; poly[c] /
  // fin[c]: chunk c's Poly1305 pass / tag check done
  hipEvent_t fork = nullptr, prep = nullptr, join = nullptr, join2 = nullptr, xdone = nullptr,
             big = nullptr;  // big: the whole-record classes done
  hipEvent_t poly[kSegChunks] = {}, fin[kSegChunks] = {};
};
struct AuxEntry {
  int dev;
  hipStream_t stream;
  AuxStream a;
};
static std::mutex g_aux_mu;
static std::vector<AuxEntry> g_aux;

static hipError_t aux_get(AuxStream *out, hipStream_t stream) {
  auto &mu = g_aux_mu;
  auto &cache = g_aux;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  for (const AuxEntry &en : cache)
    if (en.dev == dev && en.stream == stream) {
      *out = en.a;
      return hipSuccess;
    }
  AuxStream a;
  // on any failure, what was created so far is destroyed again
  auto undo = [&a]() {
    for (hipStream_t st : {a.aux, a.aux2, a.aux3})
      if (st) (void)hipStreamDestroy(st);
    for (hipEvent_t ev : {a.fork, a.prep, a.join, a.join2, a.xdone, a.big})
      if (ev) (void)hipEventDestroy(ev);
    for (int c = 0; c < kSegChunks; ++c)
      for (hipEvent_t ev : {a.poly[c], a.fin[c]})
        if (ev) (void)hipEventDestroy(ev);
  };
  for (hipStream_t *st : {&a.aux, &a.aux2, &a.aux3})
    if ((e = hipStreamCreateWithFlags(st, hipStreamNonBlocking)) != hipSuccess) {
      undo();
      return e;
    }
  for (hipEvent_t *ev : {&a.fork, &a.join, &a.prep, &a.join2, &a.xdone, &a.big})
    if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) {
      undo();
      return e;
    }
  for (int c = 0; c < kSegChunks; ++c)
    for (hipEvent_t *ev : {&a.poly[c], &a.fin[c]})
      if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) {
        undo();
        return e;
      }
  cache.push_back({dev, stream, a});
  *out = a;
  return hipSuccess;
}

static hipError_t aux_release(int dev, hipStream_t stream) {
  AuxStream a;
  bool found = false;
  {
    std::lock_guard<std::mutex> lk(g_aux_mu);
    for (size_t i = 0; i < g_aux.size(); ++i)
      if (g_aux[i].dev == dev && g_aux[i].stream == stream) {
        a = g_aux[i].a;
        g_aux.erase(g_aux.begin() + (std::ptrdiff_t)i);
        found = true;
        break;
      }
  }
  if (!found) return hipSuccess;
  hipError_t e = hipSuccess, e2;
  for (hipStream_t st : {a.aux, a.aux2, a.aux3}) {
    e2 = hipStreamSynchronize(st);
    if (e == hipSuccess) e = e2;
    e2 = hipStreamDestroy(st);
    if (e == hipSuccess) e = e2;
  }
  for (hipEvent_t ev : {a.fork, a.prep, a.join, a.join2, a.xdone, a.big}) {
    e2 = hipEventDestroy(ev);
    if (e == hipSuccess) e = e2;
  }
  for (int c = 0; c < kSegChunks; ++c)
    for (hipEvent_t ev : {a.poly[c], a.fin[c]}) {
      e2 = hipEventDestroy(ev);
      if (e == hipSuccess) e = e2;
    }
  return e;
}

// After the classifier, two branches.  Encrypt:
//   caller stream : k_seg_prep -+-> segment tile kernel (kTileSeg) --- join -> finalize
//   companion     : (fork)  the six small tile classes, the generic kernel,
//                   (wait prep) the tails (kMTTail) ---------------^
//   companion 3   : (fork)  the 2 .. 16 KiB tile classes ---------------> end
// The segment kernel is the long pole; the companion branches overlap it
// instead of following it.  The tails go last on the companion, so they
// fill the segment kernel's drain (round 2, profiles/round2/ab/; round 6:
// the tails on the idle companion 2 from the prep event were 1.5 % slower,
// profiles/round6/ab/enc_tails.md).
//
// Decrypt checks every long record's tag BEFORE any of its plaintext is
// written (crypto_aead_read, monocypher.c:2912-2929): a Poly1305 pass reads
// the ciphertext, the finalize checks the tags, then a keystream pass writes
// the plaintext of the records that verified.  The Poly1305 pass is
// HBM-bound (it moves the ciphertext once for ~15 % of the arithmetic) and
// the keystream pass VALU-bound, so the long records go through in
// kSegChunks chunks and the Poly1305 pass of chunk c + 1 runs beside the
// tag check and keystream pass of chunk c:
//   caller     : prep -> Poly(0) -(wait join)-> check(0) -> Poly(1) -> check(1) -> ...
//                ... -> check(K-1)                                   (wait xdone, join2)
//   companion  : (wait prep) tail Poly1305 -> join, small classes, generic,
//                then per chunk (wait fin[c]) the chunk's tail plaintext -> join2
//   companion 2: per chunk (wait fin[c]) XOR(c) -> xdone
// (A third companion for the tails' plaintext, so that it does not queue
// behind the small classes, measured 1-2 % slower: round 5.)
template <bool DECRYPT>
static hipError_t launch_classes(const TileArgs &ta, uint64_t nrec, const RecHdr *hdr,
                                 const uint8_t *keys, uint32_t nkeys,
                                 const noise_gpu_record *recs, const uint32_t *idx,
                                 const uint32_t *tails, const uint32_t *fin, uint64_t segbound,
                                 const uint8_t *in,
                                 uint8_t *out, const uint8_t *ad, uint8_t *status,
                                 hipStream_t stream, int chunks) {
  AuxStream ax;
  hipError_t e = aux_get(&ax, stream);
  if (e != hipSuccess) return e;
  const dim3 bt(64);
  const dim3 grid(capped((nrec + 63) / 64, NOISE_GRID_CAP));
  // a class launch: enough workgroups for the whole batch in the class (its
  // size is on the device), RPS records per super-tile -- 8 for 16 KiB, so a
  // batch of 100 K such records makes 12.5 K waves, not 1.6 K
  auto desc_grid = [nrec](uint64_t rps) { return dim3(capped((nrec + rps - 1) / rps, NOISE_GRID_CAP)); };
  SegRec *rt = const_cast<SegRec *>(ta.rt);
  // fork right after the classifier: the small classes and the generic
  // kernel need nothing else; the tails also need k_seg_prep (prep event)
  if ((e = hipEventRecord(ax.fork, stream)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(ax.aux, ax.fork, 0)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_seg_prep, grid, bt, 0, stream, keys, rt, hdr);
  if ((e = hipEventRecord(ax.prep, stream)) != hipSuccess) return e;
  TileArgs a = ta;
  const uint64_t gblocks = (nrec + kGenBlock - 1) / kGenBlock;
  const dim3 gg((unsigned)(gblocks < 2 * NOISE_GRID_CAP ? gblocks : 2 * NOISE_GRID_CAP));
  const dim3 gseg(capped((segbound + 63) / 64, NOISE_GRID_CAP));
  const dim3 gpoly(capped((segbound + 63) / 64, NOISE_GRID_CAP));
  const dim3 gxor(capped((segbound + 63) / 64, NOISE_GRID_CAP));
  const dim3 gfin(capped((nrec + 64 / NOISE_FIN_W - 1) / (64 / NOISE_FIN_W), NOISE_GRID_CAP));
  RecHdr *hdr_w = const_cast<RecHdr *>(hdr);
  // one launch per capacity: the exact-size records of the class and the
  // ragged ones of the same capacity (adjacent in idx, cls_order), the
  // masked kernel switching to its exact-size body per super-tile.  Two
  // launches per capacity (the exact tile kernel, then the masked one) left
  // nearly empty launches queued between full ones: a capped grid of single
  // -wave workgroups waits for CU slots even when it has no work (config-4
  // traces, profiles/round6/merged/cfg4_*_timeline.txt).
#define NOISE_DESC_BIG(ST)                                                     \
  NOISE_DESC_CAP(9, 16384, ST)                                                 \
  NOISE_DESC_CAP(8, 8192, ST)                                                  \
  NOISE_DESC_CAP(7, 4096, ST)                                                  \
  NOISE_DESC_CAP(6, 2048, ST)
#define NOISE_DESC_TILES()                                                     \
  NOISE_DESC_CAP(0, 64, ax.aux)                                                \
  NOISE_DESC_CAP(1, 128, ax.aux)                                               \
  NOISE_DESC_CAP(2, 192, ax.aux)                                               \
  NOISE_DESC_CAP(3, 256, ax.aux)                                               \
  NOISE_DESC_CAP(4, 512, ax.aux)                                               \
  NOISE_DESC_CAP(5, 1024, ax.aux)                                              \
  hipLaunchKernelGGL((k_aead_records<DECRYPT>), gg, dim3(kGenBlock), 0, ax.aux, keys, nkeys, recs,  \
                     nrec, idx, hdr, in, out, ad, status);
#define NOISE_DESC_CAP(C, LEN, ST)                                             \
  a.cls = C;                                                                   \
  a.cls2 = kMCls0 + C;                                                         \
  hipLaunchKernelGGL((k_aead_mtile<DECRYPT, LEN, kMTDesc>), desc_grid(MTileCfg<LEN>::RPS), bt, 0, ST, a);
  // the long records' tails (len % 1024 bytes) as masked 1 KiB tile units
  TileArgs at = a;
  at.tails = tails;
  at.ntails = &hdr->counts[kColTails];
  at.nlong = &hdr->nlong;
  at.tail_split = nullptr;
  at.chunk = -1;
  // the whole-record classes (2 .. 16 KiB) on a companion of their own, from
  // the fork: they are a quarter of config 4's bytes and would otherwise
  // queue behind (or ahead of) the small classes and the tails
  // (round 5: ahead of encrypt's segment kernel on the caller's stream
  // instead, encrypt took 5 % longer)
  if ((e = hipStreamWaitEvent(ax.aux3, ax.fork, 0)) != hipSuccess) return e;
  NOISE_DESC_BIG(ax.aux3)
  if ((e = hipEventRecord(ax.big, ax.aux3)) != hipSuccess) return e;
  if (!DECRYPT) {
    // companion: dense tile classes first, the tails (masked 1 KiB units)
    // last.  Round 6 A/B, the tails on companion 2 from the prep event
    // instead: config 4 1391-1395 against 1408-1409 GiB/s (exact lengths),
    // 1330-1336 against 1339-1351 (jittered), same box, alternating
    // (profiles/round6/ab/enc_tails.md)
    NOISE_DESC_TILES()
    if ((e = hipStreamWaitEvent(ax.aux, ax.prep, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_aead_mtile<false, 1024, kMTTail>), grid, bt, 0, ax.aux, at);
    if ((e = hipEventRecord(ax.join, ax.aux)) != hipSuccess) return e;
    // caller: every full segment of every long record, then the tags
    hipLaunchKernelGGL((k_aead_tile<DECRYPT, 1024, false, kTileSeg>), gseg, bt, 0, stream, a);
    if ((e = hipStreamWaitEvent(stream, ax.join, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_seg_finalize_w<DECRYPT, NOISE_FIN_W>), gfin, bt, 0, stream, fin, rt, ta.partial,
                       ta.partial_hi, hdr_w, in, out, status, -1);
    if ((e = hipStreamWaitEvent(stream, ax.big, 0)) != hipSuccess) return e;
    return hipGetLastError();
  }
  // decrypt.  Companion: the tails' Poly1305 first (the first tag check
  // waits for it), then the small classes and the generic kernel
  if ((e = hipStreamWaitEvent(ax.aux, ax.prep, 0)) != hipSuccess) return e;
  hipLaunchKernelGGL((k_aead_mtile<true, 1024, kMTTailPoly>), grid, bt, 0, ax.aux, at);
  if ((e = hipEventRecord(ax.join, ax.aux)) != hipSuccess) return e;
  NOISE_DESC_TILES()
  // caller: per chunk, the Poly1305 pass and the tag check (the first one
  // also waits for the tails' P_tail).  The checks sit here, not in front of
  // the keystream passes, so chunk c + 1's is done while chunk c's plaintext
  // is being written and the keystream passes follow each other without gaps
  // (one chunk: the whole range, c = -1: no split table, the finalize in the
  // classifier's bucket order)
  TileArgs ac = a;
  ac.seg_split = chunks > 1 ? hdr->ssplit : nullptr;
  auto cidx = [chunks](int c) { return chunks > 1 ? c : -1; };
  for (int c = 0; c < chunks; ++c) {
    ac.chunk = cidx(c);
    hipLaunchKernelGGL((k_aead_tile<true, 1024, false, kTileSegPoly, 0, 1, NOISE_POLY_SPAN>), gpoly, bt, 0,
                       stream, ac);
    if (c == 0 && (e = hipStreamWaitEvent(stream, ax.join, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_seg_finalize_w<true, NOISE_FIN_W>), gfin, bt, 0, stream, fin, rt, ta.partial,
                       ta.partial_hi, hdr_w, in, out, status, cidx(c));
    if ((e = hipEventRecord(ax.fin[c], stream)) != hipSuccess) return e;
  }
  // companion 2: the segments' plaintext, chunk by chunk; the companion
  // writes each chunk's tails' plaintext beside it
  for (int c = 0; c < chunks; ++c) {
    ac.chunk = cidx(c);
    if ((e = hipStreamWaitEvent(ax.aux2, ax.fin[c], 0)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_aead_tile<true, 1024, false, kTileSegXor, 0, 1, NOISE_XOR_SPAN>), gxor, bt, 0,
                       ax.aux2, ac);
    if ((e = hipStreamWaitEvent(ax.aux, ax.fin[c], 0)) != hipSuccess) return e;
    TileArgs atc = at;
    atc.chunk = cidx(c);
    atc.tail_split = chunks > 1 ? hdr->tsplit : nullptr;
    hipLaunchKernelGGL((k_aead_mtile<true, 1024, kMTTailXor>), grid, bt, 0, ax.aux, atc);
  }
#undef NOISE_DESC_CAP
#undef NOISE_DESC_TILES
#undef NOISE_DESC_BIG
  if ((e = hipEventRecord(ax.xdone, ax.aux2)) != hipSuccess) return e;
  if ((e = hipEventRecord(ax.join2, ax.aux)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(stream, ax.xdone, 0)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(stream, ax.join2, 0)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(stream, ax.big, 0)) != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t launch_aead_records(bool decrypt, const uint8_t *keys,
                               uint32_t nkeys, const noise_gpu_record *recs,
                               uint64_t nrec, const uint8_t *in, uint8_t *out,
                               const uint8_t *ad, uint8_t *status,
                               hipStream_t stream, uint64_t len_sum) {
  if (nrec == 0) return hipSuccess;
  const dim3 bg(kGenBlock);
  const uint64_t gblocks = (nrec + kGenBlock - 1) / kGenBlock;
  // Few records: the generic kernel alone (the classifier and the class
  // kernels cost ~0.13 ms per call in launches and stream joins), unless they
  // are long: one lane walks a record, ~19 us per KiB.  Same box (round 4,
  // tools/bench_small_records.py, enc + dec): 300 x 64 B 17 us generic / 262
  // classified; 300 x 1 KiB 97 / 282; 100 x 16 KiB 1909 / 353.
  const bool few = nrec < kClassifyMin && !(len_sum && len_sum / nrec >= kClassifyAvgLen);
  if (few) {
    if (decrypt)
      hipLaunchKernelGGL((k_aead_records<true>), dim3((unsigned)gblocks), bg, 0, stream, keys, nkeys, recs, nrec, nullptr, nullptr, in, out, ad, status);
    else
      hipLaunchKernelGGL((k_aead_records<false>), dim3((unsigned)gblocks), bg, 0, stream, keys, nkeys, recs, nrec, nullptr, nullptr, in, out, ad, status);
    return hipGetLastError();
  }
  if (nrec > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit indices

  // classifier geometry: at most kClsWaves waves of >= kClsMinChunk records
  uint64_t chunk = align_up((nrec + kClsWaves - 1) / kClsWaves, 64);
  if (chunk < kClsMinChunk) chunk = kClsMinChunk;
  const uint64_t nw = (nrec + chunk - 1) / chunk;
  const uint64_t segcap = nrec * 63 < kSegCapMax ? nrec * 63 : kSegCapMax;

  // scratch: header | part[nw][kCols] | wbase[nw][kCols] | idx[nrec] |
  //          tails[nrec] | fin[nrec] | rt[nrec] | segs[segcap] | partial[segcap] |
  //          partial_hi[segcap]
  const uint64_t o_part = sizeof(RecHdr);
  const uint64_t o_wbase = align_up(o_part + nw * kCols * 4, 256);
  const uint64_t o_idx = align_up(o_wbase + nw * kCols * 8, 256);
  const uint64_t o_tails = align_up(o_idx + nrec * 4, 256);
  const uint64_t o_fin = align_up(o_tails + nrec * 4, 256);
  const uint64_t o_rt = align_up(o_fin + nrec * 4, 256);
  const uint64_t o_segs = align_up(o_rt + nrec * sizeof(SegRec), 256);
  const uint64_t o_part2 = align_up(o_segs + segcap * sizeof(SegEntry), 256);
  const uint64_t o_phi = align_up(o_part2 + segcap * sizeof(SegPartial), 256);
  const uint64_t bytes = o_phi + segcap * sizeof(uint32_t);
  void *mem = nullptr;
  hipError_t e = scratch_get(&mem, bytes, stream);
  if (e != hipSuccess) return e;
  uint8_t *base = static_cast<uint8_t *>(mem);
  RecHdr *hdr = reinterpret_cast<RecHdr *>(base);
  uint32_t *part = reinterpret_cast<uint32_t *>(base + o_part);
  unsigned long long *wbase = reinterpret_cast<unsigned long long *>(base + o_wbase);
  uint32_t *idx = reinterpret_cast<uint32_t *>(base + o_idx);
  uint32_t *tails = reinterpret_cast<uint32_t *>(base + o_tails);
  uint32_t *fin = reinterpret_cast<uint32_t *>(base + o_fin);
  SegRec *rt = reinterpret_cast<SegRec *>(base + o_rt);
  SegEntry *segs = reinterpret_cast<SegEntry *>(base + o_segs);
  SegPartial *partial = reinterpret_cast<SegPartial *>(base + o_part2);
  uint32_t *partial_hi = reinterpret_cast<uint32_t *>(base + o_phi);

  const dim3 b64(64);
  hipLaunchKernelGGL(k_cls_count, dim3((unsigned)nw), b64, 0, stream, recs, nrec, (uint32_t)chunk, keys, nkeys, in, out, part);
  hipLaunchKernelGGL(k_cls_scan, dim3(kCols), b64, 0, stream, part, (uint32_t)nw, wbase, hdr, segcap);
  hipLaunchKernelGGL(k_cls_scatter, dim3((unsigned)nw), b64, 0, stream, recs, nrec, (uint32_t)chunk, keys, nkeys, in, out, wbase, hdr, idx, rt, segs, tails, fin, segcap);

  TileArgs ta{};
  ta.in = in;
  ta.out = out;
  ta.status = status;
  ta.keys = keys;
  ta.nkeys = nkeys;
  ta.recs = recs;
  ta.idx = idx;
  ta.cls_base = hdr->cls_base;
  ta.counts = hdr->counts;
  ta.segs = segs;
  ta.rt = rt;
  ta.partial = partial;
  ta.partial_hi = partial_hi;
  ta.nseg = &hdr->nseg;
  // the decrypt pipeline's chunks pay off on large batches only (each chunk
  // adds four launches and a stream hand-off)
  const int chunks = nrec >= kChunkMinRecords ? kSegChunks : 1;
  return decrypt ? launch_classes<true>(ta, nrec, hdr, keys, nkeys, recs, idx, tails, fin, segcap,
                                       in, out, ad, status, stream, chunks)
                 : launch_classes<false>(ta, nrec, hdr, keys, nkeys, recs, idx, tails, fin, segcap,
                                         in, out, ad, status, stream, 1);
}

}  // namespace noise_amd
