// unit_kernel.hpp -- verify-first decrypt of long records, one wave per
// "unit" of whole records, streamed twice through a 16 KiB LDS window
// (records_kernels.hip, round 5).
//
// Noise decrypt must check a record's tag before any of its plaintext leaves
// (crypto_aead_read, monocypher.c:2912-2929).  The segment path does that
// with a Poly1305 pass over every long record, a tag-check kernel, then a
// keystream pass, in chunks over three streams: the ciphertext is read twice
// ~1 GB apart, and the passes' launches, hand-offs and latency-bound tag
// checks sit between them.  Here one wave owns a unit of whole records
// (<= 64 items of 1 KiB) and runs the three steps back to back:
//   P. the unit's items pass through the wave's 16-slot LDS window, a quarter
//      (16 items) at a time: Poly1305 of the ciphertext -> P per item (LDS);
//   T. every record of the unit: Horner over its items' P in R = r^64, then
//      * r^tb + P_tail, the length block, the tag, compared -> status, verdict;
//   X. the quarters again (the second read follows the first within the
//      wave's own unit, ~64 KiB later, while the unit's lines are still in
//      the caches): keystream, and the plaintext of verified records only
//      (a failed record: zeros out of place, nothing in place).
// No workgroup barrier and no cross-wave hand-off: the window holds one
// quarter, so the other waves on the SIMD cover each quarter's DMA wait.
//
// Units.  A long record (1024 < len <= 65535, 16-byte aligned, AD-free) has
// m = nfull + (len % 1024 != 0) items: its full 1 KiB segments and its tail.
// The classifier sorts long records into buckets b = floor(log2(m - 1)) (m
// in 2 | 3-4 | 5-8 | 9-16 | 17-32 | 33-64), and a unit is k_b = 32 >> b
// records of one bucket: at most k_b * 2^(b+1) = 64 items.  Units run largest
// bucket first.  Item slot s of a unit: the S full segments first, then the T
// tails; quarter w holds slots 16w .. 16w + 15.
#pragma once
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kUnitItems = 64;   // 1 KiB items per unit
constexpr int kUnitBuckets = 6;

// the bucket of a long record with m = nfull + (tail != 0) items (2..64)
__host__ __device__ constexpr int unit_bucket(uint32_t m) {
  return 31 - __builtin_clz((m - 1u) | 1u);
}

struct UnitArgs {
  const uint8_t *in;
  uint8_t *out;
  uint8_t *status;                         // per descriptor
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
// r^(16 m), m = 0..3, from the SegRec (m = 0: 1)
__device__ __forceinline__ F26 seg_pow16(const SegRec &R, uint32_t m) {
  const uint32_t mi = m ? m - 1u : 0u;
  const uint4 v = *reinterpret_cast<const uint4 *>(R.pwlo[mi]);
  const uint32_t v4 = R.pwhi[mi];
  F26 f;
  f.a[0] = m ? v.x : 1u; f.a[1] = m ? v.y : 0u; f.a[2] = m ? v.z : 0u;
  f.a[3] = m ? v.w : 0u; f.a[4] = m ? v4 : 0u;
  return f;
}
// f * (use ? y : 1), with the same instructions either way
__device__ __forceinline__ F26 mul26_if(const F26 &f, const F26 &y, bool use) {
  F26 s;
#pragma unroll
  for (int i = 0; i < 5; ++i) s.a[i] = use ? y.a[i] : (i == 0 ? 1u : 0u);
  return mul26(f, s);
}
__device__ __forceinline__ void poly_key(Poly1305 &p, const uint32_t r[4]) {
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
  p.r0 = r[0]; p.r1 = r[1]; p.r2 = r[2]; p.r3 = r[3];
  p.rr0 = (p.r0 >> 2) * 5u;
  p.rr1 = p.r1 + (p.r1 >> 2);
  p.rr2 = p.r2 + (p.r2 >> 2);
  p.rr3 = p.r3 + (p.r3 >> 2);
  p.r0lo = p.r0 & 3u;
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

// quarter w of the unit, from lane r's record (q, len) (r < nrec): segment
// slots 16w .. 16w + 15 (lane: slot 16w + lane / 4) and the quarter's tails
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

// HBM -> the LDS window: quarter w's segments (one LDS-DMA instruction each,
// the tile kernel's swizzle) and tails (window slot S + t_lo + tt - 16w).
// The piece holding a record's last bytes ends inside its tag, so every
// ciphertext piece is whole.
__device__ __forceinline__ void unit_dma(const uint8_t *in, uint4 *win, const UnitMap &m, uint32_t w,
                                         const uint32_t gl[4], uint64_t in_rec, uint64_t tin_rec,
                                         uint32_t lane) {
  const uint64_t io = in_rec + 1024ull * m.js, tio = tin_rec + 1024ull * m.nft;
  const uint32_t in_lo = (uint32_t)io, in_hi = (uint32_t)(io >> 32);
  const uint32_t tin_lo = (uint32_t)tio, tin_hi = (uint32_t)(tio >> 32);
  // (wave-uniform; readfirstlane keeps the compiler from a VGPR M0 base)
  const uint32_t nv = uniform32(m.nv), nt = uniform32(m.nt), t0 = uniform32(m.S + m.t_lo - 16u * w);
#pragma unroll
  for (int qq = 0; qq < 16; ++qq) {
    if ((uint32_t)qq < nv) {
      const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)in_hi, 4 * qq),
                                  (uint32_t)__builtin_amdgcn_readlane((int)in_lo, 4 * qq));
      lds_dma16_s<true>(in + off, 16u * glq<256>(gl, qq), (lds_void *)(NOISE_LDS3(win) + 64 * qq));
    }
  }
#pragma unroll 1
  for (uint32_t tt = 0; tt < nt; ++tt) {
    const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)tin_hi, (int)tt),
                                (uint32_t)__builtin_amdgcn_readlane((int)tin_lo, (int)tt));
    const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane((int)m.tlt, (int)tt);
    uint4 *slot = win + 64u * (t0 + tt);
    // (the LDS-DMA writes lane l's 16 bytes to M0 + 16 l: slot + lane)
    if (16u * lane < tb) lds_dma16_v<true>(in + off + 16u * lane, (lds_void *)NOISE_LDS3(slot));
  }
}

// One wave per unit (grid-stride over the units).  Every load of a step is
// issued before its one wait, and every load is unconditional from a valid
// SegRec (lanes without a segment or tail read some lane's record; the
// values are used only where valid): a load inside a branch would be waited
// for at the branch's end, the window's DMA included.
__global__ __launch_bounds__(64) void k_unit_dec(const UnitArgs a) {
  __shared__ uint4 win[16 * 64];              // the window: one quarter's 16 item slots
  __shared__ uint32_t part[kUnitItems * 5];   // P per item of the unit: words h0..h4
  __shared__ uint32_t okf[32];                // record r of the unit verified
  using C = TileCfg<1024, 256>;               // a segment: 4 lanes x 256 B
  const uint32_t lane = threadIdx.x;
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
  uint32_t gl[4];  // swz(64q + lane) - 64q (tile_kernel.hpp)
#pragma unroll
  for (int i = 0; i < 4; ++i) gl[i] = swz<256>(64u * i + lane) - 64u * i;
  const uint32_t rho = lane >> 2, j4 = lane & 3u;        // segment lanes: 4 per segment
  const uint32_t tg = lane >> 4, ti = lane & 15u;        // tail lanes: 16 per tail, 4 tails a round

#pragma unroll 1
  for (uint64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
    const UnitPlace pl = unit_place(u, units, cnt, fbase);
    const uint32_t nrec = pl.nrec;
    const uint64_t f = lane < nrec ? pl.p0 + lane : pl.p0;
    const uint32_t q = a.fin[f], len = a.finl[f];
    const UnitMap m0 = unit_map(q, len, nrec, nlong, 0u, lane);
    const uint32_t nq = uniform32((m0.S + m0.T + 15u) >> 4);  // quarters with items

    // ---- P. Poly1305 over the ciphertext, a quarter at a time --------------
#pragma unroll 1
    for (uint32_t w = 0; w < nq; ++w) {
      const UnitMap m = unit_map(q, len, nrec, nlong, w, lane);
      uint64_t in_rec, tin_rec;
      uint32_t sr[4];
      F26 spw;
      {
        const SegRec &R = a.rt[m.qs];
        in_rec = R.in_off;
#pragma unroll
        for (int k = 0; k < 4; ++k) sr[k] = R.r[k];
        spw = seg_pow16(R, 3u - j4);  // r^(16 (3 - j4)): the lane's recombination weight
      }
      tin_rec = a.rt[m.qt].in_off;
      unit_dma(a.in, win, m, w, gl, in_rec, tin_rec, lane);
      // the first tail round's key material (lands with the DMA)
      uint32_t tr0[4];
      F26 tp16, tp32;
      {
        const uint32_t tq0 = (uint32_t)__shfl((int)m.qt, (int)(tg < m.nt ? tg : 0u));
        const SegRec &R = a.rt[tq0];
#pragma unroll
        for (int k = 0; k < 4; ++k) tr0[k] = R.r[k];
        tp16 = seg_pow16(R, 1u);
        tp32 = seg_pow16(R, 2u);
      }
      wait_vmem();
      wave_lds_fence();
      if (m.nv) {
        Poly1305 p;
        poly_key(p, sr);
#pragma unroll
        for (int kk = 0; kk < C::CPL; ++kk) {
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {
            const uint4 v = win[swz<256>(rho * C::SPR + 4u * (j4 * C::CPL + kk) + qd)];
            poly_block(p, v.x, v.y, v.z, v.w);
          }
        }
        // lane j4's 16-block sum * r^(16 (3 - j4)), summed over the 4 lanes
        F26 h = mul26(to26(p.h0, p.h1, p.h2, p.h3, p.h4), spw);
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
          uint32_t *pp = part + 5u * (16u * w + rho);
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
        if (tr) {  // rounds after the first (units of many short records)
          const SegRec &R = a.rt[qr];
#pragma unroll
          for (int k = 0; k < 4; ++k) tr0[k] = R.r[k];
          tp16 = seg_pow16(R, 1u);
          tp32 = seg_pow16(R, 2u);
        }
        Poly1305 p;
        poly_key(p, tr0);
        const uint4 *slot = win + 64u * (m.S + m.t_lo + src - 16u * w) + 4u * ti;
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
          F26 pw = to26(p.r0, p.r1, p.r2, p.r3, 0u);  // r^1, r^2, r^4, r^8 by squaring
          h = mul26_if(h, pw, (e & 1u) != 0u);
          pw = mul26(pw, pw);
          h = mul26_if(h, pw, (e & 2u) != 0u);
          pw = mul26(pw, pw);
          h = mul26_if(h, pw, (e & 4u) != 0u);
          pw = mul26(pw, pw);
          h = mul26_if(h, pw, (e & 8u) != 0u);
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
          uint32_t *pp = part + 5u * (m.S + m.t_lo + tt);
          pp[0] = h0; pp[1] = h1; pp[2] = h2; pp[3] = h3; pp[4] = h4;
        }
      }
      // the window's reads done before the next quarter's DMA overwrites it;
      // the partial sums written before T reads them
      wait_lds();
      wave_lds_fence();
    }

    // ---- T. every record of the unit: the tag, checked --------------------
    // record g: W lanes (nf <= W: W = 64 / np2(nrec) >= 2^(b+1)), lane ii
    // takes the record's segment ii
    {
      uint32_t np2 = 1;
      while (np2 < nrec) np2 <<= 1;
      const uint32_t W = 64u / np2, logW = 31u - (uint32_t)__builtin_clz(W);
      const uint32_t g = lane >> logW, ii = lane & (W - 1u);
      const uint32_t gs = g < nrec ? g : 0u;
      const uint32_t qg = (uint32_t)__shfl((int)q, (int)gs);
      const uint32_t nfg = (uint32_t)__shfl((int)m0.nf, (int)gs);
      const uint32_t tlg = (uint32_t)__shfl((int)m0.tl, (int)gs);
      const uint32_t lg = (uint32_t)__shfl((int)len, (int)gs);
      const uint32_t seg0 = (uint32_t)__shfl((int)m0.incl, (int)gs) - nfg;
      const uint32_t tslot = m0.S + (uint32_t)__shfl((int)m0.tincl, (int)gs) - 1u;
      const bool act = g < nrec && nfg != 0u;
      F26 rp;  // R = r^64, then its squares
      uint32_t fr[4], fs[4], fdi;
      uint64_t f_in;
      F26 frt;
      {
        const SegRec &R = a.rt[qg];
        rp = f26_load(R.r64);
#pragma unroll
        for (int k = 0; k < 4; ++k) { fr[k] = R.r[k]; fs[k] = R.s[k]; }
        fdi = R.di;
        f_in = R.in_off;
        frt = f26_load(R.rtail);
      }
      // the received tag (byte loads: every lane reads a valid record's)
      const uint4 want = load16<false>(a.in + f_in + lg, 16);
      F26 acc = {{0u, 0u, 0u, 0u, 0u}};
      if (act && ii < nfg) {
        const uint32_t *pp = part + 5u * (seg0 + ii);
        acc = to26(pp[0], pp[1], pp[2], pp[3], pp[4]);
      }
      const uint32_t e = nfg > ii ? nfg - 1u - ii : 0u;  // 0..62
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        acc = mul26_if(acc, rp, ((e >> b) & 1u) != 0u);
        if (b < 5) rp = mul26(rp, rp);
      }
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
          const uint32_t *pp = part + 5u * tslot;
          const F26 v = to26(pp[0], pp[1], pp[2], pp[3], pp[4]);
#pragma unroll
          for (int k = 0; k < 5; ++k) acc.a[k] += v.a[k];
        }
        carry26(acc);
        carry26(acc);
        Poly1305 p;
        poly_key(p, fr);
        from26(acc, p.h0, p.h1, p.h2, p.h3, p.h4);
        p.s0 = fs[0]; p.s1 = fs[1]; p.s2 = fs[2]; p.s3 = fs[3];
        poly_block(p, 0u, 0u, lg, 0u);  // LE64(ad_len = 0) || LE64(len)
        uint32_t tag[4];
        poly_final(p, tag);
        const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) |
                              (want.w ^ tag[3]);
        a.status[fdi] = diff == 0u ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
        okf[g] = diff == 0u ? 1u : 0u;
      }
      // the verdicts are LDS writes of this wave (in order); the fence keeps
      // the compiler -- and the CPU emulator's lanes, which are threads --
      // from moving the reads in X before them
      wait_lds();
      wave_lds_fence();
    }

    // ---- X. keystream, verified plaintext -> HBM, a quarter at a time -----
#pragma unroll 1
    for (uint32_t w = 0; w < nq; ++w) {
      const UnitMap m = unit_map(q, len, nrec, nlong, w, lane);
      uint64_t s_in, s_out, t_in, t_out, nonce;
      uint32_t kt[8];
      {
        const SegRec &R = a.rt[m.qs];
        s_in = R.in_off;
        s_out = R.out_off;
        nonce = R.nonce;
#pragma unroll
        for (int k = 0; k < 8; ++k) kt[k] = R.k[k];
      }
      {
        const SegRec &R = a.rt[m.qt];
        t_in = R.in_off;
        t_out = R.out_off;
      }
      unit_dma(a.in, win, m, w, gl, s_in, t_in, lane);
      uint32_t tk[8];
      uint64_t tnonce;
      {
        const uint32_t tq0 = (uint32_t)__shfl((int)m.qt, (int)(tg < m.nt ? tg : 0u));
        const SegRec &R = a.rt[tq0];
#pragma unroll
        for (int k = 0; k < 8; ++k) tk[k] = R.k[k];
        tnonce = R.nonce;
      }
      wait_vmem();
      wave_lds_fence();
      if (m.nv) {
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
            const uint4 v = win[slot];
            // a lane past the quarter's segments leaves its slot alone: it
            // may hold one of the unit's tails
            if (m.sv) win[slot] = make_uint4(v.x ^ ks[4 * qd + 0], v.y ^ ks[4 * qd + 1],
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
        uint4 *slot = win + 64u * (m.S + m.t_lo + src - 16u * w) + 4u * ti;
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
      // the stores read other lanes' slots: every lane's XOR first
      wait_lds();
      wave_lds_fence();
      const uint64_t oo = s_out + 1024ull * m.js, too = t_out + 1024ull * m.nft;
      const uint32_t out_lo = (uint32_t)oo, out_hi = (uint32_t)(oo >> 32);
      const uint32_t tout_lo = (uint32_t)too, tout_hi = (uint32_t)(too >> 32);
      const uint32_t inpl = a.in + s_in == a.out + s_out, tinpl = a.in + t_in == a.out + t_out;
#pragma unroll
      for (int qq = 0; qq < 16; ++qq) {
        if ((uint32_t)qq < m.nv) {
          const uint4 v = win[swz<256>(64u * qq + lane)];
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
        const uint4 v = ok ? win[64u * (m.S + m.t_lo + tt - 16u * w) + lane] : make_uint4(0u, 0u, 0u, 0u);
        const int rem = (int)tb - (int)(16u * lane);
        uint8_t *dst = a.out + off + 16u * lane;
        if ((ok || !ip) && rem >= 16) store16<true>(dst, v, 16);
        else if ((ok || !ip) && rem > 0) store16<false>(dst, v, rem);
      }
      // the window's reads done before the next quarter's (or unit's) DMA
      wait_lds();
      wave_lds_fence();
    }
  }
}

}  // namespace noise_amd
