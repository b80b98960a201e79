// unit_kernel.hpp -- long records as whole-record "units" held in LDS
// (records_kernels.hip, round 5).
//
// Why: Noise decrypt must check a record's tag before any of its plaintext
// leaves (crypto_aead_read, monocypher.c:2912-2929).  With long records cut
// into 1 KiB segments spread over the whole GPU, that meant a Poly1305 pass
// over the ciphertext, a tag check, then a keystream pass that read the
// ciphertext from HBM a second time (round 4: 1.61x the algorithmic traffic,
// decrypt 15 % slower than encrypt).  Here a 4-wave workgroup owns whole
// records: it moves a unit of them (<= 64 KiB) into LDS once, computes the
// keystream and Poly1305 in one pass over the LDS image (the plaintext stays
// in LDS), checks every tag inside the workgroup, and only then stores the
// verified records.  One HBM read and one write per byte, in both directions.
//
// Units.  A long record (1024 < len <= 65535, 16-byte aligned, AD-free) has
// m = nfull + (len % 1024 != 0) items: its full 1 KiB segments and its tail.
// The classifier sorts long records into buckets b = floor(log2(m - 1)) (m
// in 2 | 3-4 | 5-8 | 9-16 | 17-32 | 33-64), and a unit is k_b = 32 >> b
// records of one bucket: at most k_b * 2^(b+1) = 64 items, more than 32 when
// the bucket is full, exactly 64 for power-of-two lengths (BASELINE config 4).
// Units run largest bucket first.
//
// LDS: 64 item slots of 1 KiB.  The unit's S full segments take slots
// 0..S-1, its T tails slots S..S+T-1; wave w owns slots 16w..16w+15, moves
// them in (one LDS-DMA instruction per segment, the tile kernel's swizzle)
// and out, and computes them:
//   * segments: the tile kernel's fused 1 KiB work unit (4 lanes x 256 B,
//     ChaCha20 + Poly1305 Horner in the clamped r, recombination by r^16,
//     r^32) -> the segment's Poly1305 sum P_s = sum_i m_i r^(64-i);
//   * tails: 16 lanes per tail, lane i the tail's 64-byte chunk i (one ChaCha
//     block, <= 4 Poly1305 blocks, bytes past the record masked), weighted by
//     r^(tb - end_i) and summed -> P_tail = sum_b m_b r^(tb-b) (tb: the tail's
//     Poly1305 blocks);
// then, after a workgroup barrier, wave 0 combines each record (W lanes per
// record, Horner over its P_s in R = r^64, then * r^tb + P_tail, the length
// block, poly_final), stores (encrypt) or checks (decrypt) the tag, and after
// a second barrier every wave stores its slots: the ciphertext, or the
// plaintext of verified records only (a failed record: zeros out of place,
// nothing in place -- what the tile and lane paths do).
#pragma once
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kUnitWaves = 4;
constexpr int kUnitThreads = 64 * kUnitWaves;
constexpr int kUnitItems = 64;               // 1 KiB item slots per unit
constexpr int kUnitSlots = 64 * kUnitItems;  // 16-byte LDS slots (64 KiB)
constexpr int kUnitBuckets = 6;

// the bucket of a long record with m = nfull + (tail != 0) items (2..64)
__device__ __forceinline__ int unit_bucket(uint32_t m) {
  return 31 - __builtin_clz((m - 1u) | 1u);
}

struct UnitArgs {
  const uint8_t *in;
  uint8_t *out;
  uint8_t *status;                         // decrypt: per descriptor
  const SegRec *rt;                        // k_seg_prep: key, nonce, r, s, powers
  const uint32_t *fin;                     // long records by bucket (classifier)
  const uint32_t *finl;                    // their lengths, in the same order
  const unsigned long long *bucket_cnt;    // [kUnitBuckets] records per bucket
  const unsigned long long *nlong;         // records with a SegRec (q < nlong)
};

// wave-wide inclusive prefix sum (all 64 lanes participate)
__device__ __forceinline__ uint32_t unit_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl((int)v, (int)(lane >= (uint32_t)d ? lane - d : lane));
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}
// the first lane whose (non-decreasing) inclusive count exceeds x
__device__ __forceinline__ uint32_t unit_find(uint32_t incl, uint32_t x) {
  uint32_t lo = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1) {
    const uint32_t probe = (uint32_t)__shfl((int)incl, (int)(lo + step - 1));
    if (probe <= x) lo += step;
  }
  return lo;
}

__device__ __forceinline__ F26 f26_load(const uint32_t *w) {
  F26 f;
#pragma unroll
  for (int i = 0; i < 5; ++i) f.a[i] = w[i];
  return f;
}
// f * (use ? y : 1), with the same instructions either way
__device__ __forceinline__ F26 mul26_if(const F26 &f, const F26 &y, bool use) {
  F26 s;
#pragma unroll
  for (int i = 0; i < 5; ++i) s.a[i] = use ? y.a[i] : (i == 0 ? 1u : 0u);
  return mul26(f, s);
}

// where unit u's records are: fin[p0 .. p0 + nrec) (buckets largest first)
struct UnitPlace {
  uint64_t p0;
  uint32_t nrec;
};
__device__ __forceinline__ UnitPlace unit_place(uint64_t u, const uint64_t units[kUnitBuckets],
                                                const uint64_t cnt[kUnitBuckets],
                                                const uint64_t fbase[kUnitBuckets]) {
  int b = kUnitBuckets - 1;
  uint64_t i = u;
#pragma unroll
  for (int bb = kUnitBuckets - 1; bb > 0; --bb) {
    if (b == bb && i >= units[bb]) {
      i -= units[bb];
      b = bb - 1;
    }
  }
  UnitPlace pl{0, 0};
#pragma unroll
  for (int bb = 0; bb < kUnitBuckets; ++bb)
    if (bb == b) {
      const uint64_t kb = 32u >> bb, left = cnt[bb] - i * kb;
      pl.p0 = fbase[bb] + i * kb;
      pl.nrec = (uint32_t)(left < kb ? left : kb);
    }
  return pl;
}

// the unit's slot map, from lane r's record (q, len) (r < nrec): wave w's
// segment slots 16w .. 16w + 15 (lane: slot 16w + lane / 4) and its tails
struct UnitMap {
  uint32_t nf, tl, incl, tincl;  // lane r: record r
  uint32_t S, T, nv, t_lo, nt;   // wave-uniform
  uint32_t rs, qs, js;           // lane: its segment's record (in the unit, q), segment number
  bool sv;
  uint32_t rt, qt, tlt, nft;     // lane < nt: tail t_lo + lane's record, q, bytes, full segments
};
__device__ __forceinline__ UnitMap unit_map(uint32_t q, uint32_t len, uint32_t nrec, uint64_t nlong,
                                            uint32_t w, uint32_t lane) {
  UnitMap m;
  const bool has = lane < nrec && q < nlong;  // q >= nlong: beyond the SegRec table (generic)
  m.nf = has ? len >> 10 : 0u;
  m.tl = has ? len & 1023u : 0u;
  m.incl = unit_scan(m.nf, lane);
  m.S = (uint32_t)__builtin_amdgcn_readlane((int)m.incl, 63);
  m.tincl = unit_scan(m.tl ? 1u : 0u, lane);
  m.T = (uint32_t)__builtin_amdgcn_readlane((int)m.tincl, 63);
  const uint32_t x = 16u * w + (lane >> 2);
  m.nv = m.S > 16u * w ? (m.S - 16u * w < 16u ? m.S - 16u * w : 16u) : 0u;
  m.rs = unit_find(m.incl, x) & 63u;
  m.qs = (uint32_t)__shfl((int)q, (int)m.rs);
  m.js = x - ((uint32_t)__shfl((int)m.incl, (int)m.rs) - (uint32_t)__shfl((int)m.nf, (int)m.rs));
  m.sv = x < m.S;
  const int t_lo_i = (int)(16u * w) - (int)m.S;
  m.t_lo = t_lo_i > 0 ? (uint32_t)t_lo_i : 0u;
  const uint32_t t_hi_c = 16u * w + 16u > m.S ? 16u * w + 16u - m.S : 0u;
  const uint32_t t_hi = t_hi_c < m.T ? t_hi_c : m.T;
  m.nt = t_hi > m.t_lo ? t_hi - m.t_lo : 0u;
  m.rt = unit_find(m.tincl, m.t_lo + lane) & 63u;
  m.qt = (uint32_t)__shfl((int)q, (int)m.rt);
  m.tlt = (uint32_t)__shfl((int)m.tl, (int)m.rt);
  m.nft = (uint32_t)__shfl((int)m.nf, (int)m.rt);
  return m;
}

// HBM -> LDS: wave w's segments (one LDS-DMA instruction each, the tile
// kernel's swizzle) and tails.  The piece holding a record's last bytes ends
// inside its tag, so every ciphertext piece is whole.
__device__ __forceinline__ void unit_dma(const uint8_t *in, uint4 *img, uint4 *wimg, const UnitMap &m,
                                         const uint32_t gl[4], uint64_t in_rec, uint64_t tin_rec,
                                         uint32_t lane) {
  const uint64_t io = in_rec + 1024ull * m.js, tio = tin_rec + 1024ull * m.nft;
  const uint32_t in_lo = (uint32_t)io, in_hi = (uint32_t)(io >> 32);
  const uint32_t tin_lo = (uint32_t)tio, tin_hi = (uint32_t)(tio >> 32);
  // (wave-uniform; readfirstlane keeps the compiler from a VGPR M0 base
  // after the next unit's map went through a branch)
  const uint32_t nv = uniform32(m.nv), nt = uniform32(m.nt), t0 = uniform32(m.S + m.t_lo);
#pragma unroll
  for (int qq = 0; qq < 16; ++qq) {
    if ((uint32_t)qq < nv) {
      const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)in_hi, 4 * qq),
                                  (uint32_t)__builtin_amdgcn_readlane((int)in_lo, 4 * qq));
      lds_dma16_s<true>(in + off, 16u * glq<256>(gl, qq), (lds_void *)(NOISE_LDS3(wimg) + 64 * qq));
    }
  }
#pragma unroll 1
  for (uint32_t tt = 0; tt < nt; ++tt) {
    const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)tin_hi, (int)tt),
                                (uint32_t)__builtin_amdgcn_readlane((int)tin_lo, (int)tt));
    const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane((int)m.tlt, (int)tt);
    uint4 *slot = img + 64u * (t0 + tt);
    // (the LDS-DMA writes lane l's 16 bytes to M0 + 16 l: slot + lane)
    if (16u * lane < tb) lds_dma16_v<true>(in + off + 16u * lane, (lds_void *)NOISE_LDS3(slot));
  }
}
// the record offsets of the lane's segment and tail (unit_dma adds the
// segment's position: nothing uses the loaded words before then, so the
// loads are waited for only where the DMA needs them)
__device__ __forceinline__ void unit_in_addr(const UnitArgs &a, const UnitMap &m, uint32_t lane,
                                             uint64_t &in_rec, uint64_t &tin_rec) {
  in_rec = tin_rec = 0u;
  if (m.sv) in_rec = a.rt[m.qs].in_off;
  if (lane < m.nt) tin_rec = a.rt[m.qt].in_off;
}

// NOISE_UNIT_STAMPS (timing builds only, tools/unit_ab.py): per-phase
// s_memrealtime sums over every wave, read by noise_amd_unit_stamps()
#if defined(NOISE_UNIT_STAMPS) && !defined(NOISE_HIP_EMU)
__device__ unsigned long long g_unit_ts[8];
#define UNIT_TS(i)                                                   \
  do {                                                               \
    const uint64_t t_ = __builtin_amdgcn_s_memrealtime();            \
    ts_acc[i] += t_ - ts_last;                                       \
    ts_last = t_;                                                    \
  } while (0)
#else
#define UNIT_TS(i) ((void)0)
#endif

// Decrypt, per unit, wave w (one workgroup barrier per unit; the loop is
// software-pipelined: the unit's ciphertext is already on its way into LDS
// when an iteration starts):
//   A. the metadata of the unit's segments, tails and of the records this
//      wave checks (records w, w + 4, ...: r^64 powers, r, s, r^tb, the
//      received tag), and the next unit's record list -- loads that land
//      with the DMA;
//   C. Poly1305 over the ciphertext in LDS -> P per item (double-buffered by
//      unit parity: a wave that runs ahead into the next unit cannot
//      overwrite partial sums a slower wave still reads);
//   -- __syncthreads: every P of the unit is in LDS --
//   D. the wave's records: W lanes per record, lane i takes segment i,
//      P_i R^(nf-1-i) (six selected products, R^(2^b) from k_seg_prep),
//      summed; * r^tb + P_tail, the length block, the tag, compared with the
//      received one -> status and a verdict in LDS; then an LDS counter;
//   E. the next unit's slot map and ciphertext addresses (loads), then the
//      keystream: plaintext into LDS (while the other waves check tags);
//   F. once every wave's verdicts are in (the counter), the verified records'
//      plaintext to HBM (a failed record: zeros out of place, nothing in
//      place), then at once the next unit's DMA into the freed slots.
__global__ __launch_bounds__(kUnitThreads, 2) void k_unit_dec(const UnitArgs a) {
  __shared__ uint4 img[kUnitSlots];              // the unit's item slots
  __shared__ uint32_t part[2][kUnitItems * 5];   // P per item, by unit parity: words h0..h4
  __shared__ uint32_t okf[32];                   // record r of the unit verified
  __shared__ uint32_t fdone;                     // waves done checking: 4 per unit
  using C = TileCfg<1024, 256>;                  // a segment: 4 lanes x 256 B
  // w, S, T and everything derived from them are wave-uniform: readfirstlane
  // keeps them in SGPRs (the LDS-DMA's M0 base must be one)
  const uint32_t lane = threadIdx.x & 63u, w = uniform32(threadIdx.x >> 6);
  if (threadIdx.x == 0) fdone = 0u;  // ordered before any add by the first unit's barrier
  const uint64_t nlong = *a.nlong;
  uint64_t cnt[kUnitBuckets], units[kUnitBuckets], fbase[kUnitBuckets], nunits = 0;
  {
    uint64_t b0 = 0;
#pragma unroll
    for (int b = 0; b < kUnitBuckets; ++b) {
      cnt[b] = a.bucket_cnt[b];
      fbase[b] = b0;
      b0 += cnt[b];
      const uint64_t k = 32u >> b;
      units[b] = (cnt[b] + k - 1) / k;
      nunits += units[b];
    }
  }
  uint64_t u = blockIdx.x;
  if (u >= nunits) return;
  uint32_t gl[4];  // swz(64q + lane) - 64q (tile_kernel.hpp)
#pragma unroll
  for (int i = 0; i < 4; ++i) gl[i] = swz<256>(64u * i + lane) - 64u * i;
  uint4 *wimg = img + 1024u * w;  // this wave's 16 slots
  // prologue: the first unit's records and its DMA
  UnitPlace pl = unit_place(u, units, cnt, fbase);
  uint32_t q = 0, len = 0;
  if (lane < pl.nrec) {
    q = a.fin[pl.p0 + lane];
    len = a.finl[pl.p0 + lane];
  }
  {
    const UnitMap m = unit_map(q, len, pl.nrec, nlong, w, lane);
    uint64_t in_rec, tin_rec;
    unit_in_addr(a, m, lane, in_rec, tin_rec);
    unit_dma(a.in, img, wimg, m, gl, in_rec, tin_rec, lane);
  }
  uint32_t it = 0;  // units done by this workgroup
#if defined(NOISE_UNIT_STAMPS) && !defined(NOISE_HIP_EMU)
  uint64_t ts_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t ts_last = __builtin_amdgcn_s_memrealtime();
#endif

#pragma unroll 1
  for (;;) {
    ++it;
    uint32_t *pt = part[it & 1u];
    const UnitMap m = unit_map(q, len, pl.nrec, nlong, w, lane);
    const uint32_t nrec = pl.nrec;
    // ---- A. metadata (lands with the DMA issued at the end of the last unit).
    // Loads only: nothing below uses a loaded word before the one wait, so
    // they all travel together with the DMA instead of one after another.
    // the next unit's records first (past the last unit: fin[0], never used)
    const uint64_t u2 = u + gridDim.x;
    const bool has2 = u2 < nunits;
    UnitPlace pl2{0, 0};
    if (has2) pl2 = unit_place(u2, units, cnt, fbase);
    const uint64_t f2 = lane < pl2.nrec ? pl2.p0 + lane : 0u;
    const uint32_t q2 = a.fin[f2], len2 = a.finl[f2];
    // (Every load is unconditional, from a valid SegRec -- lanes without a
    // segment or tail read record qs / qt of some lane -- and the values are
    // only used where they are valid: a load inside a branch would be waited
    // for at the branch's end, the DMA in front of it included.)
    uint32_t sr[4], kt[8];
    uint64_t nonce, s_in, s_out;
    F26 pw16, pw32;
    {
      const SegRec &R = a.rt[m.qs];
      s_in = R.in_off;
      s_out = R.out_off;
      nonce = R.nonce;
#pragma unroll
      for (int k = 0; k < 8; ++k) kt[k] = R.k[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) sr[k] = R.r[k];
      pw16 = f26_load(R.pw16);
      pw32 = f26_load(R.pw32);
    }
    uint64_t t_in, t_out;
    {
      const SegRec &R = a.rt[m.qt];
      t_in = R.in_off;
      t_out = R.out_off;
    }
    // the first tail round's Poly1305 inputs (lane: tail tg of the round)
    const uint32_t tg = lane >> 4, ti = lane & 15u;
    uint32_t tr0[4];
    F26 tp8, tp16, tp32;
    const uint32_t tq0 = (uint32_t)__shfl((int)m.qt, (int)(tg < m.nt ? tg : 0u));
    {
      const SegRec &R = a.rt[tq0];
#pragma unroll
      for (int k = 0; k < 4; ++k) tr0[k] = R.r[k];
      tp8 = f26_load(R.pw8);
      tp16 = f26_load(R.pw16);
      tp32 = f26_load(R.pw32);
    }
    // the records this wave checks: g = w + 4 gi, W lanes each, lane ii
    // takes the record's segment ii (nf <= W always: W = 8 2^b >= 2^(b+1))
    const uint32_t nrw = nrec > w ? (nrec - w + 3u) >> 2 : 0u;
    uint32_t np2 = 1;
    while (np2 < nrw) np2 <<= 1;
    const uint32_t W = 64u / np2, logW = 31u - (uint32_t)__builtin_clz(W);
    const uint32_t gi = lane >> logW, ii = lane & (W - 1u), g = w + 4u * gi;
    const uint32_t gs = gi < nrw ? g : 0u;
    const uint32_t qg = (uint32_t)__shfl((int)q, (int)gs);
    const uint32_t nfg = (uint32_t)__shfl((int)m.nf, (int)gs);
    const uint32_t tlg = (uint32_t)__shfl((int)m.tl, (int)gs);
    const uint32_t lg = (uint32_t)__shfl((int)len, (int)gs);
    const uint32_t seg0 = (uint32_t)__shfl((int)m.incl, (int)gs) - nfg;
    const uint32_t tslot = m.S + (uint32_t)__shfl((int)m.tincl, (int)gs) - 1u;
    const bool act = gi < nrw && nfg != 0u;
    F26 rp0, rp1, rp2, rp3, rp4, rp5;  // R^(2^b)
    uint32_t fr[4], fs[4], fdi;
    uint64_t f_in;
    F26 frt;
    {
      const SegRec &R = a.rt[qg];
      rp0 = f26_load(R.r64);
      rp1 = f26_load(R.rpow[0]);
      rp2 = f26_load(R.rpow[1]);
      rp3 = f26_load(R.rpow[2]);
      rp4 = f26_load(R.rpow[3]);
      rp5 = f26_load(R.rpow[4]);
#pragma unroll
      for (int k = 0; k < 4; ++k) { fr[k] = R.r[k]; fs[k] = R.s[k]; }
      fdi = R.di;
      f_in = R.in_off;
      frt = f26_load(R.rtail);
    }
    wait_vmem();
    wave_lds_fence();
    UNIT_TS(0);
    // the received tags (needed in D: their latency hides behind C; byte
    // loads, unconditional -- every lane reads a valid record's tag -- so
    // that nothing waits for them before D)
    const uint4 want = load16<false>(a.in + f_in + lg, 16);

    // ---- C. Poly1305 over the ciphertext ------------------------------------
    if (m.nv) {
      Poly1305 p;
      p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
      p.r0 = sr[0]; p.r1 = sr[1]; p.r2 = sr[2]; p.r3 = sr[3];
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      const uint32_t rho = lane >> 2, j4 = lane & 3u;
#pragma unroll
      for (int kk = 0; kk < C::CPL; ++kk) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const uint4 v = wimg[swz<256>(rho * C::SPR + 4u * (j4 * C::CPL + kk) + qd)];
          poly_block(p, v.x, v.y, v.z, v.w);
        }
      }
      // lane j4's 16-block sum * r^(16 (3 - j4)), summed over the 4 lanes
      F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
      const uint32_t mm = 3u - j4;
      h = mul26_if(h, pw16, (mm & 1u) != 0u);
      h = mul26_if(h, pw32, (mm & 2u) != 0u);
#pragma unroll
      for (int bt = 0; bt < 2; ++bt) {
#pragma unroll
        for (int k = 0; k < 5; ++k) h.a[k] += __shfl_xor(h.a[k], 1 << bt);
      }
      carry26(h);
      carry26(h);
      uint32_t h0, h1, h2, h3, h4;
      from26(h, h0, h1, h2, h3, h4);
      if (m.sv && j4 == 0u) {
        uint32_t *pp = pt + 5u * (16u * w + rho);
        pp[0] = h0; pp[1] = h1; pp[2] = h2; pp[3] = h3; pp[4] = h4;
      }
    }
    // tails: 16 lanes per tail (four per round), lane ti the tail's 64-byte
    // chunk ti: its <= 4 blocks (bytes past the record masked), then
    // * r^(tb - end) where its chain ended at block end
#pragma unroll 1
    for (uint32_t tr = 0; tr < m.nt; tr += 4u) {
      const uint32_t tt = tr + tg;
      const bool tv = tt < m.nt;
      const uint32_t src = tv ? tt : 0u;
      const uint32_t qr = (uint32_t)__shfl((int)m.qt, (int)src);
      const uint32_t tb = (uint32_t)__shfl((int)m.tlt, (int)src);  // tail bytes
      if (tr) {  // rounds after the first (units of many short records): load here
        const SegRec &R = a.rt[qr];
#pragma unroll
        for (int k = 0; k < 4; ++k) tr0[k] = R.r[k];
        tp8 = f26_load(R.pw8);
        tp16 = f26_load(R.pw16);
        tp32 = f26_load(R.pw32);
      }
      Poly1305 p;
      p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
      p.r0 = tr0[0]; p.r1 = tr0[1]; p.r2 = tr0[2]; p.r3 = tr0[3];
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      const uint4 *slot = img + 64u * (m.S + m.t_lo + (tv ? tt : 0u)) + 4u * ti;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int rem = (int)tb - (int)(16u * (4u * ti + qd));
        if (tv && rem > 0) {
          const uint4 vm = mask_bytes(slot[qd], rem >= 16 ? 16 : rem);
          poly_block(p, vm.x, vm.y, vm.z, vm.w);
        }
      }
      const uint32_t nbt = (tb + 15u) >> 4;
      const uint32_t end = 4u * ti + 4u < nbt ? 4u * ti + 4u : nbt;
      const uint32_t e = nbt > end ? nbt - end : 0u;  // 0..60
      F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
      {
        F26 pw = to26(p.r0, p.r1, p.r2, p.r3, 0u);  // r^1, r^2, r^4 by squaring
        h = mul26_if(h, pw, (e & 1u) != 0u);
        pw = mul26(pw, pw);
        h = mul26_if(h, pw, (e & 2u) != 0u);
        pw = mul26(pw, pw);
        h = mul26_if(h, pw, (e & 4u) != 0u);
        h = mul26_if(h, tp8, (e & 8u) != 0u);
        h = mul26_if(h, tp16, (e & 16u) != 0u);
        h = mul26_if(h, tp32, (e & 32u) != 0u);
      }
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
        for (int k = 0; k < 5; ++k) h.a[k] += __shfl_xor(h.a[k], 1 << bt);
      }
      carry26(h);
      carry26(h);
      uint32_t h0, h1, h2, h3, h4;
      from26(h, h0, h1, h2, h3, h4);
      if (tv && ti == 0u) {
        uint32_t *pp = pt + 5u * (m.S + m.t_lo + tt);
        pp[0] = h0; pp[1] = h1; pp[2] = h2; pp[3] = h3; pp[4] = h4;
      }
    }
    UNIT_TS(1);
    __syncthreads();
    UNIT_TS(2);

    // ---- D. this wave's records: the tag, checked ----------------------------
    // (the status byte is stored in F: a global store here would be waited
    // for by the next memory instruction's count, at the start of E)
    uint32_t st_rec = 0xffu;
    if (nrw) {
      F26 acc = {{0u, 0u, 0u, 0u, 0u}};
      if (act && ii < nfg) {
        const uint32_t *pp = pt + 5u * (seg0 + ii);
        acc = to26(pp[0], pp[1], pp[2], pp[3], pp[4]);
      }
      const uint32_t e = nfg > ii ? nfg - 1u - ii : 0u;  // 0..62
      acc = mul26_if(acc, rp0, (e & 1u) != 0u);
      acc = mul26_if(acc, rp1, (e & 2u) != 0u);
      acc = mul26_if(acc, rp2, (e & 4u) != 0u);
      acc = mul26_if(acc, rp3, (e & 8u) != 0u);
      acc = mul26_if(acc, rp4, (e & 16u) != 0u);
      acc = mul26_if(acc, rp5, (e & 32u) != 0u);
      // limbs < 2^26 + 2^9: 16 of them fit in 32 bits, 64 do not
#pragma unroll
      for (int bt = 0; bt < 6; ++bt) {
        if ((uint32_t)bt < logW) {
          if (bt == 4) carry26(acc);
#pragma unroll
          for (int k = 0; k < 5; ++k) acc.a[k] += (uint32_t)__shfl_xor((int)acc.a[k], 1 << bt);
        }
      }
      if (act && ii == 0u) {
        if (tlg) {
          carry26(acc);
          acc = mul26(acc, frt);
          const uint32_t *pp = pt + 5u * tslot;
          const F26 v = to26(pp[0], pp[1], pp[2], pp[3], pp[4]);
#pragma unroll
          for (int k = 0; k < 5; ++k) acc.a[k] += v.a[k];
        }
        carry26(acc);
        carry26(acc);
        Poly1305 p;
        from26(acc, p.h0, p.h1, p.h2, p.h3, p.h4);
        p.r0 = fr[0]; p.r1 = fr[1]; p.r2 = fr[2]; p.r3 = fr[3];
        p.rr0 = (p.r0 >> 2) * 5u;
        p.rr1 = p.r1 + (p.r1 >> 2);
        p.rr2 = p.r2 + (p.r2 >> 2);
        p.rr3 = p.r3 + (p.r3 >> 2);
        p.r0lo = p.r0 & 3u;
        p.s0 = fs[0]; p.s1 = fs[1]; p.s2 = fs[2]; p.s3 = fs[3];
        poly_block(p, 0u, 0u, lg, 0u);  // LE64(ad_len = 0) || LE64(len)
        uint32_t tag[4];
        poly_final(p, tag);
        const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) |
                              (want.w ^ tag[3]);
        st_rec = diff == 0u ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;  // stored in F
        okf[g] = diff == 0u ? 1u : 0u;
      }
    }
    // this wave's verdicts are in LDS (LDS operations of a wave complete in
    // order; the fence keeps the compiler -- and the CPU emulator's lanes,
    // which are threads -- from moving lane 0's add before them)
    // The hand-off is LDS-only: a release-ordered add would also wait for
    // the global status store above (vmcnt(0), ~2-3 us on the checking wave's
    // critical path: measured); the verdicts are LDS writes of this wave,
    // done once lgkmcnt reaches 0.
    wait_lds();
    wave_lds_fence();
    if (lane == 0) __hip_atomic_fetch_add(&fdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    UNIT_TS(3);

    // ---- E. the next unit's addresses (loads), the keystream -----------------
    // the first tail round's key and nonce (their latency hides behind the
    // segments' keystream)
    uint32_t tk[8];
    uint64_t tnonce;
    {
      const SegRec &R = a.rt[tq0];
#pragma unroll
      for (int k = 0; k < 8; ++k) tk[k] = R.k[k];
      tnonce = R.nonce;
    }
    UnitMap m2 = m;
    uint64_t n_in_rec = 0, n_tin_rec = 0;
    if (has2) {
      m2 = unit_map(q2, len2, pl2.nrec, nlong, w, lane);
      unit_in_addr(a, m2, lane, n_in_rec, n_tin_rec);
    }
    if (m.nv) {
      const uint32_t rho = lane >> 2, j4 = lane & 3u;
      const uint32_t c0 = j4 * C::CPL;
      const uint32_t cb = 1u + 16u * m.js + c0;
      const uint32_t n_lo = (uint32_t)nonce, n_hi = (uint32_t)(nonce >> 32);
      const ChaPre pre = chacha_pre(kt, n_lo, n_hi);
      uint32_t ks[16];
      chacha20_block_pre(kt, cb, pre, n_lo, n_hi, ks);
#pragma unroll
      for (int kk = 0; kk < C::CPL; ++kk) {
        const uint32_t c = c0 + kk;
        uint32_t ksn[16];
        if (kk + 1 < C::CPL) chacha20_block_pre(kt, cb + 1u + kk, pre, n_lo, n_hi, ksn);
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const uint32_t slot = swz<256>(rho * C::SPR + 4u * c + qd);
          const uint4 v = wimg[slot];
          // a lane past the wave's segments leaves its slot alone: it may be
          // one of the unit's tails
          if (m.sv) wimg[slot] = make_uint4(v.x ^ ks[4 * qd + 0], v.y ^ ks[4 * qd + 1],
                                            v.z ^ ks[4 * qd + 2], v.w ^ ks[4 * qd + 3]);
        }
        if (kk + 1 < C::CPL) {
#pragma unroll
          for (int k = 0; k < 16; ++k) ks[k] = ksn[k];
        }
      }
    }
#pragma unroll 1
    for (uint32_t tr = 0; tr < m.nt; tr += 4u) {
      const uint32_t tt = tr + tg;
      const bool tv = tt < m.nt;
      const uint32_t src = tv ? tt : 0u;
      const uint32_t qr = (uint32_t)__shfl((int)m.qt, (int)src);
      const uint32_t tb = (uint32_t)__shfl((int)m.tlt, (int)src);
      const uint32_t nfr = (uint32_t)__shfl((int)m.nft, (int)src);
      if (tr) {
        const SegRec &R = a.rt[qr];
#pragma unroll
        for (int k = 0; k < 8; ++k) tk[k] = R.k[k];
        tnonce = R.nonce;
      }
      uint32_t ks[16];
      chacha20_block(tk, 1u + 16u * nfr + ti, (uint32_t)tnonce, (uint32_t)(tnonce >> 32), ks);
      uint4 *slot = img + 64u * (m.S + m.t_lo + (tv ? tt : 0u)) + 4u * ti;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int rem = (int)tb - (int)(16u * (4u * ti + qd));
        if (tv && rem > 0) {
          const uint4 v = slot[qd];
          slot[qd] = mask_bytes(make_uint4(v.x ^ ks[4 * qd + 0], v.y ^ ks[4 * qd + 1],
                                           v.z ^ ks[4 * qd + 2], v.w ^ ks[4 * qd + 3]),
                                rem >= 16 ? 16 : rem);
        }
      }
    }

    // ---- F. every verdict of the unit in: the verified plaintext -> HBM ------
    // (the stores read other lanes' slots: every lane's keystream XOR first)
    wave_lds_fence();
    UNIT_TS(4);
    while (__hip_atomic_load(&fdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4u * it)
      __builtin_amdgcn_s_sleep(1);
    wave_lds_fence();  // the verdict reads below stay after the counter (LDS, in order)
    wait_vmem();  // the next unit's addresses (long landed): nothing but stores after this
    UNIT_TS(5);
    if (st_rec != 0xffu) a.status[fdi] = (uint8_t)st_rec;
    const uint64_t oo = s_out + 1024ull * m.js, too = t_out + 1024ull * m.nft;
    const uint32_t out_lo = (uint32_t)oo, out_hi = (uint32_t)(oo >> 32);
    const uint32_t tout_lo = (uint32_t)too, tout_hi = (uint32_t)(too >> 32);
    const uint32_t inpl = a.in + s_in == a.out + s_out, tinpl = a.in + t_in == a.out + t_out;
#pragma unroll
    for (int qq = 0; qq < 16; ++qq) {
      if ((uint32_t)qq < m.nv) {
        const uint4 v = wimg[swz<256>(64u * qq + lane)];
        const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)m.rs, 4 * qq);
        const bool ok = okf[r] != 0u;
        const bool ip = __builtin_amdgcn_readlane((int)inpl, 4 * qq) != 0;
        const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)out_hi, 4 * qq),
                                    (uint32_t)__builtin_amdgcn_readlane((int)out_lo, 4 * qq));
        if (ok) store16<true>(a.out + off + 16u * lane, v, 16);
        else if (!ip) store16<true>(a.out + off + 16u * lane, make_uint4(0u, 0u, 0u, 0u), 16);
      }
    }
#pragma unroll 1
    for (uint32_t tt = 0; tt < m.nt; ++tt) {
      const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)m.rt, (int)tt);
      const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane((int)m.tlt, (int)tt);
      const bool ok = okf[r] != 0u;
      const bool ip = __builtin_amdgcn_readlane((int)tinpl, (int)tt) != 0;
      const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)tout_hi, (int)tt),
                                  (uint32_t)__builtin_amdgcn_readlane((int)tout_lo, (int)tt));
      const uint4 v = ok ? img[64u * (m.S + m.t_lo + tt) + lane] : make_uint4(0u, 0u, 0u, 0u);
      const int rem = (int)tb - (int)(16u * lane);
      uint8_t *dst = a.out + off + 16u * lane;
      if ((ok || !ip) && rem >= 16) store16<true>(dst, v, 16);
      else if ((ok || !ip) && rem > 0) store16<false>(dst, v, rem);
    }
    if (!has2) break;
    // the next unit's DMAs overwrite these slots: the reads above are done
    wait_lds();
    wave_lds_fence();
    unit_dma(a.in, img, wimg, m2, gl, n_in_rec, n_tin_rec, lane);
    UNIT_TS(6);
    u = u2;
    pl = pl2;
    q = q2;
    len = len2;
  }
#if defined(NOISE_UNIT_STAMPS) && !defined(NOISE_HIP_EMU)
  ts_acc[7] = it;
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_unit_ts[i], (unsigned long long)ts_acc[i]);
#endif
}

}  // namespace noise_amd
