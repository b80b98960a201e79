// mtile_kernel.hpp -- the masked ("ragged") tile kernel: the LDS-staged AEAD
// of tile_kernel.hpp for records of ANY length 1 <= len <= L in a tile class
// of capacity L (the fast paths were keyed to a
// fixed table of lengths; 1000-, 1400- or 5000-byte records fell to a lane
// per record).  Same reference semantics: crypto_aead_write / _read
// (monocypher.c:2899-2929) under the Noise nonce 0^32 || LE64(n)
// (noise.cpp:207-215), any length (noise.cpp:202-281).
//
// Layout: the record's bytes sit in the tile at their own (16-byte aligned)
// positions, as for an exact record; only the lanes' view is shifted.  A
// class of capacity L has CV = L / 64 ChaCha chunk slots per record, G lanes
// of CPL chunks each.  A record of C = ceil(len / 64) chunks is RIGHT-aligned
// in them: lane j's virtual chunk v is real chunk CPL j + v - (CV - C), absent
// when negative -- the absent chunks are LEADING ones.  The MAC of a lane
// starts from h = 0, so resetting h to 0 after each absent chunk makes them
// vanish, and every lane keeps the exact-size weight r^(BPL (G-1-j)): the
// recombination is tile_kernel.hpp's, unchanged, with no per-record powers.
// The loop is tile_kernel.hpp's too: one LDS read of a piece feeds the XOR
// and the MAC, and the ChaCha block of chunk k + 1 is computed beside the
// XOR / MAC of chunk k.  Only the record's last chunk (lane G-1's last) is
// special: its MAC input is masked to the record's bytes (the AEAD's zero
// padding: no tag bytes, keystream or stale tile bytes), and its blocks past
// P = ceil(len / 16) multiply by r = 1 with no 2^128 bit -- identities.
// The tag sits at byte len: it is read out of (decrypt) / shifted into
// (encrypt) the two 16-byte pieces it straddles.  Stores: the whole 16-byte
// pieces of the output, then the partial last piece (dword / short / byte
// stores) -- no byte past the record's output is written (len + 16 encrypt,
// len decrypt; Noise wire ct || tag).
//
// Reads: the 16-byte aligned pieces holding the record's input bytes are
// read whole.  A record starts 16-byte aligned (the callers check it), so the
// last piece ends at most 15 bytes past the input and never crosses a page:
// those bytes (padding, a neighbour's, the in-place tag) are masked, never
// used or written.
//
// Modes (MT_*):
//   kMTUniform   one key, nonce0 + i, record i at in + i * in_stride (strides
//                and bases 16-byte aligned), len = a.len
//   kMTDesc      descriptor records of one ceiling class (records_kernels.hip)
//   kMTTail      the tail (len % 1024 bytes past the full 1 KiB segments) of
//                a long record, encrypt: ciphertext + its Poly1305 sum P_tail
//                into the SegRec, no tag (k_seg_finalize_w adds the rest)
//   kMTTailPoly  decrypt, before the tags are known: P_tail of the ciphertext
//   kMTTailXor   decrypt, after k_seg_finalize_w: plaintext of the tails of
//                the records whose tag verified (a failed one: nothing in
//                place, zeros as a copy)
// The tail modes read r, r^16, r^32 and the key from the record's SegRec
// (k_seg_prep) instead of a key pass; ChaCha counters continue at 1 + 16 nf.
#pragma once
#include <type_traits>

#include "tile_kernel.hpp"

namespace noise_amd {

// two waves per SIMD (<= 256 VGPRs): the masked kernels hold more state
// than the exact ones and the compiler would otherwise take AGPRs and drop
// to one wave per SIMD (the CPU emulation build has no such attribute)
#if defined(NOISE_HIP_EMU)
#define NOISE_OCC2
#else
#define NOISE_OCC2 __attribute__((amdgpu_waves_per_eu(2)))
#endif

enum MTileMode : int { kMTUniform = 0, kMTDesc = 1, kMTTail = 2, kMTTailPoly = 3, kMTTailXor = 4 };

// 16 bytes at byte offset k (1..15) of the 32-byte little-endian [lo | hi].
// The word shift by k / 4 (0..3) is two v_perm word selects per word (a
// plain select of w[i + 2] / w[i] is turned into a scratch-indexed load by
// the compiler), then a byte funnel (v_alignbyte).
__device__ __forceinline__ uint32_t wsel(uint32_t sel, uint32_t a, uint32_t b) {
  return __builtin_amdgcn_perm(a, b, sel);  // sel 0x07060504: a, 0x03020100: b
}
__device__ __forceinline__ uint4 extract16(const uint4 lo, const uint4 hi, uint32_t k) {
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t s8 = (k & 8u) ? 0x07060504u : 0x03020100u, s4 = (k & 4u) ? 0x07060504u : 0x03020100u;
  uint32_t u[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) u[i] = wsel(s8, w[i + 2], w[i]);
  uint32_t v[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) v[i] = wsel(s4, u[i + 1], u[i]);
  const uint32_t b = k & 3u;
  uint4 o;
  o.x = __builtin_amdgcn_alignbyte(v[1], v[0], b);
  o.y = __builtin_amdgcn_alignbyte(v[2], v[1], b);
  o.z = __builtin_amdgcn_alignbyte(v[3], v[2], b);
  o.w = __builtin_amdgcn_alignbyte(v[4], v[3], b);
  return o;
}

// Poly1305 block with explicit r values: (r = 1, rr = 0, r0lo = 1, hb = 0,
// m = 0) leaves h unchanged (partially reduced) -- a trailing absent block
__device__ __forceinline__ void poly_block_r(Poly1305 &p, uint32_t m0, uint32_t m1, uint32_t m2,
                                             uint32_t m3, uint32_t hb, uint32_t r0, uint32_t r1,
                                             uint32_t r2, uint32_t r3, uint32_t rr0, uint32_t rr1,
                                             uint32_t rr2, uint32_t rr3, uint32_t r0lo) {
  unsigned c;
  const uint32_t s0 = __builtin_addc(p.h0, m0, 0u, &c);
  const uint32_t s1 = __builtin_addc(p.h1, m1, c, &c);
  const uint32_t s2 = __builtin_addc(p.h2, m2, c, &c);
  const uint32_t s3 = __builtin_addc(p.h3, m3, c, &c);
  const uint32_t s4 = p.h4 + c + hb;
  const uint64_t x0 = mad64(s0, r0, mad64(s1, rr3, mad64(s2, rr2, mad64(s3, rr1, mad64(s4, rr0, 0)))));
  const uint64_t x1 = mad64(s0, r1, mad64(s1, r0, mad64(s2, rr3, mad64(s3, rr2, mad64(s4, rr1, 0)))));
  const uint64_t x2 = mad64(s0, r2, mad64(s1, r1, mad64(s2, r0, mad64(s3, rr3, mad64(s4, rr2, 0)))));
  const uint64_t x3 = mad64(s0, r3, mad64(s1, r2, mad64(s2, r1, mad64(s3, r0, mad64(s4, rr3, 0)))));
  const uint32_t x4 = __umul24(s4, r0lo);
  const uint32_t u5 = x4 + (uint32_t)(x3 >> 32);
  const uint32_t q = u5 >> 2;
  p.h0 = __builtin_addc(q + (q << 2), (uint32_t)x0, 0u, &c);
  p.h1 = __builtin_addc((uint32_t)x1, (uint32_t)(x0 >> 32), c, &c);
  p.h2 = __builtin_addc((uint32_t)x2, (uint32_t)(x1 >> 32), c, &c);
  p.h3 = __builtin_addc((uint32_t)x3, (uint32_t)(x2 >> 32), c, &c);
  p.h4 = (u5 & 3u) + c;
}

// The first `n` (1..15) bytes of a 16-byte piece at a 16-byte aligned
// address: whole dwords, then a short and a byte as needed
__device__ __forceinline__ void store_head(uint8_t *p, uint4 v, uint32_t n) {
#if defined(NOISE_HIP_EMU)
  store16<false>(p, v, (int)n);  // the emulator's store hook sees it as one store
#else
  typedef __attribute__((address_space(1))) uint32_t g_u32;
  typedef __attribute__((address_space(1))) uint16_t g_u16;
  typedef __attribute__((address_space(1))) uint8_t g_u8;
  g_u32 *p32 = (g_u32 *)p;
  if (n >= 4u) p32[0] = v.x;
  if (n >= 8u) p32[1] = v.y;
  if (n >= 12u) p32[2] = v.z;
  const uint32_t q = n >> 2, rem = n & 3u;
  const uint32_t last = q == 0u ? v.x : q == 1u ? v.y : q == 2u ? v.z : v.w;
  uint8_t *t = p + 4u * q;
  if (rem & 2u) *(g_u16 *)t = (uint16_t)last;
  if (rem & 1u) *(g_u8 *)(t + (rem & 2u)) = (uint8_t)(last >> (8u * (rem & 2u)));
#endif
}

// Tile shape of capacity L (a multiple of 64).  Up to 7 chunks (448 B): one
// lane per record, CPL = L / 64.  Above: lanes of 4 chunks (256 B), G = L / 256
// lanes per record -- G need not divide 64 (1280 B: G = 5, 12 records on 60
// lanes; lanes past RPT G idle), which gives capacities between the powers of
// two (the uniform dispatch, aead_kernels.hip).
template <int L>
struct MTileCfg {
  static constexpr int NCH = L / 64;
  static constexpr int G = NCH <= 7 ? 1 : NCH / 4;
  static constexpr int CPL = NCH / G;
  static constexpr int BPL = 4 * CPL;
  static constexpr int RPT = 64 / G;
  static constexpr int LANES = RPT * G;  // working lanes
  static constexpr int SPR = L / 16;
  static constexpr int S = 4 * CPL;      // slots of one lane's span
  static constexpr int REC_SLOTS = RPT * SPR;
  static constexpr int NSLOT = REC_SLOTS + RPT;
  static constexpr int LOG2G = G <= 1 ? 0 : G <= 2 ? 1 : G <= 4 ? 2 : G <= 8 ? 3 : G <= 16 ? 4 : G <= 32 ? 5 : 6;
  // records per super-tile (one key lane each): 64, at most 128 KiB for
  // capacities above 2 KiB (batches of large records make waves), a
  // multiple of RPT
  static constexpr int RPS0 = L > 2048 ? 64 * 2048 / L : 64;
  static constexpr int RPS = RPS0 >= RPT ? RPS0 / RPT * RPT : RPT;
  static_assert(L % 64 == 0 && L >= 64 && L <= 16384 && (NCH <= 7 || NCH % 4 == 0), "capacity");
};

// slot of piece g (lane spans of S slots; pieces of a span stay in it).
// Spans of 4, 8, 16 slots: swz<256> (conflict-free ds_read_b128).  12, 20,
// 24, 28 (one lane of 3, 5, 6, 7 chunks): swz<256> is 3-4-way conflicted
// there, so the span is rotated by k(l) = (l >> 2) & 3 ((l >> 1) & 7 for 24):
// the 16 lanes of a read group then hit 16 distinct bank quads.
template <int S>
__device__ __forceinline__ uint32_t rot_k(uint32_t l) {
  return S == 24 ? (l >> 1) & 7u : (l >> 2) & 3u;
}
template <int S>
__device__ __forceinline__ uint32_t mslot(uint32_t g) {
  if constexpr (S == 4 || S == 8 || S == 16) {
    return swz<256>(g);
  } else {
    const uint32_t l = g / S, i = g % S, t = i + rot_k<S>(l);
    return (uint32_t)S * l + (t >= (uint32_t)S ? t - S : t);
  }
}
// piece held by slot s (mslot's inverse)
template <int S>
__device__ __forceinline__ uint32_t mpiece(uint32_t s) {
  if constexpr (S == 4 || S == 8 || S == 16) {
    return swz<256>(s);
  } else {
    const uint32_t l = s / S, i = s % S, t = i + (uint32_t)S - rot_k<S>(l);
    return (uint32_t)S * l + (t >= (uint32_t)S ? t - S : t);
  }
}

template <bool DECRYPT, int L, int MODE>
__global__ __launch_bounds__(64) NOISE_OCC2 void k_aead_mtile(const TileArgs a) {
  using C = MTileCfg<L>;
  constexpr int G = C::G, CPL = C::CPL, BPL = C::BPL, SPR = C::SPR, RPT = C::RPT, S = C::S;
  constexpr int REC_SLOTS = C::REC_SLOTS, NSLOT = C::NSLOT;
  constexpr bool IDLE = C::LANES < 64;  // lanes past RPT G do no work
  constexpr int ZSLOT = NSLOT, JSLOT = NSLOT + 1;  // zero slot, junk slot (absent XOR writes)
  constexpr bool TAIL = MODE >= kMTTail;
  constexpr bool KEYED = MODE != kMTUniform;
  constexpr bool DO_XOR = MODE != kMTTailPoly;
  constexpr bool DO_POLY = MODE != kMTTailXor;
  constexpr bool TAG_IN = DECRYPT && !TAIL;   // input ct || tag, check the tag
  constexpr bool TAG_OUT = !DECRYPT && !TAIL; // output ct || tag
  constexpr bool POLY_PRE = DECRYPT;          // Poly1305 over the input (before the XOR)
  static_assert(!TAIL || L == 1024, "tails are cut to 1 KiB units");
  static_assert(MODE != kMTTail || !DECRYPT, "the fused tail pass is encrypt's");
  static_assert(MODE < kMTTailPoly || DECRYPT, "the split tail passes are decrypt's");
  constexpr int OPR = TAG_OUT ? SPR + 1 : SPR;  // output pieces of a full record
  constexpr int KPR = SPR / 64;                 // KiB per record (L >= 1024)
  constexpr bool WHOLE_KIB = SPR % 64 == 0;
  static_assert(!WHOLE_KIB || S == 16, "whole-KiB records: lane spans of 16 slots");
  // 256 / 512-byte classes: a DMA or store instruction covers RPI = 64 / SPR
  // (4, 2) whole records -- their lengths and offsets come from RPI
  // v_readlanes and a per-lane select instead of a shuffle per piece (the
  // uniform mode computes them per lane: no shuffles to save)
  constexpr bool SUB_KIB = KEYED && (SPR == 16 || SPR == 32);
  static_assert(!SUB_KIB || S == 16, "256 / 512-byte records: lane spans of 16 slots");
  constexpr int RPI = SUB_KIB ? 64 / SPR : 1;
  // records per super-tile: 64 (one key lane each), at most 128 KiB for
  // classes of 4 KiB and up (so that batches of large records make waves)
  constexpr int RPS = C::RPS;
  constexpr int NTS = RPS / RPT;
  static_assert(NTS >= 1 && RPS % RPT == 0, "super-tile shape");
  __shared__ uint4 lds[NSLOT + 2];
  uint4 *lb = lds;
  const uint32_t lane = threadIdx.x;
  // idle lanes (past RPT G) shadow record 0: they read its tile, write the
  // junk slot, and are never valid
  const uint32_t rho = lane < (uint32_t)C::LANES ? lane / G : 0u, j = lane % G;
  const bool idle = IDLE && lane >= (uint32_t)C::LANES;
  if (lane == 0) lds[ZSLOT] = make_uint4(0u, 0u, 0u, 0u);  // never overwritten
  // mtab[n]: the mask keeping the first n (0..16) bytes of a 16-byte piece
  __shared__ uint4 mtab[17];
  if (lane <= 16u) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = (int)lane - 4 * i;
      w[i] = b >= 4 ? 0xffffffffu : b <= 0 ? 0u : (1u << (8 * b)) - 1u;
    }
    mtab[lane] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  wave_lds_fence();
  uint32_t gl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) gl[i] = swz<256>(64u * i + lane) - 64u * i;

  // the work list
  uint64_t nrec = a.nrec, dbase = 0;
  if (MODE == kMTDesc) {
    // the exact-size records of the capacity, then the ragged ones (adjacent
    // in idx: k_cls_scatter); a super-tile of exact ones only takes the
    // exact-size body below
    dbase = a.cls_base[a.cls];
    nrec = a.counts[a.cls] + (a.cls2 >= 0 ? a.counts[a.cls2] : 0ull);
  } else if (TAIL) {
    const uint64_t nall = *a.ntails;
    uint64_t lo = 0, hi = nall;
    if (a.chunk >= 0 && a.tail_split) {
      lo = a.tail_split[a.chunk] < nall ? a.tail_split[a.chunk] : nall;
      hi = a.tail_split[a.chunk + 1] < nall ? a.tail_split[a.chunk + 1] : nall;
    }
    dbase = lo;
    nrec = hi > lo ? hi - lo : 0;
  }
  const uint64_t nlong = TAIL ? *a.nlong : 0ull;
  uint32_t kuni[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) kuni[i] = a.key.w[i];
  const uint8_t *in = a.in;
  uint8_t *out = a.out;

#pragma unroll 1
  for (uint64_t super0 = (uint64_t)blockIdx.x * RPS; super0 < nrec;
       super0 += (uint64_t)gridDim.x * RPS) {
    // ---- key pass: lane l -> record super0 + l --------------------------
    uint32_t own_k[8], own_nlo = 0, own_nhi = 0, own_len = 0, own_cb = 0, own_di = 0, own_q = 0;
    uint32_t own_in_lo = 0, own_in_hi = 0, own_out_lo = 0, own_out_hi = 0;
    bool own_bad = false, own_inplace = false, own_ok = true;
    uint32_t kr[4] = {0u, 0u, 0u, 0u}, kss[4] = {0u, 0u, 0u, 0u};
    F26 own_rt;  // r^(16 - t) (G > 1; from the SegRec for the tails)
#pragma unroll
    for (int i = 0; i < 5; ++i) own_rt.a[i] = 0u;
    F26 pw[C::LOG2G > 0 ? C::LOG2G : 1];
#pragma unroll
    for (int b = 0; b < (C::LOG2G > 0 ? C::LOG2G : 1); ++b)
#pragma unroll
      for (int i = 0; i < 5; ++i) pw[b].a[i] = 0u;
    {
      const uint64_t rec = super0 + lane;
      const bool have = rec < nrec && lane < (uint32_t)RPS;
      uint64_t n = 0, ioff = 0, ooff = 0;
      uint32_t ki = 0;
      if (MODE == kMTUniform) {
        n = a.nonce0 + rec;
        ioff = rec * a.in_stride;
        ooff = rec * a.out_stride;
        own_len = have ? a.len : 0u;
      } else if (MODE == kMTDesc) {
        if (have) {
          own_di = a.idx[dbase + rec];
          const noise_gpu_record d = a.recs[own_di];
          ki = d.key_idx;
          n = d.nonce;
          ioff = d.in_off;
          ooff = d.out_off;
          own_len = d.len;
        }
      } else {  // tails: the long record's SegRec
        if (have) {
          own_q = a.tails[dbase + rec];
          if (own_q < nlong) {
            const SegRec &R = a.rt[own_q];
            const uint32_t nf = R.nfull;
            n = R.nonce;
            ioff = R.in_off + 1024ull * nf;
            ooff = R.out_off + 1024ull * nf;
            own_len = R.len - 1024u * nf;
            own_cb = 16u * nf;
            if (MODE == kMTTailXor) own_ok = R.ok != 0u;
#pragma unroll
            for (int i = 0; i < 8; ++i) own_k[i] = R.k[i];
            if (DO_POLY) {
#pragma unroll
              for (int i = 0; i < 4; ++i) kr[i] = R.r[i];
              // G = 4 lanes: r^16, r^32, and r^(16 - t) of the tail (k_seg_prep)
#pragma unroll
              for (int b = 0; b < C::LOG2G; ++b) {
                pw[b].a[0] = R.pwlo[b][0]; pw[b].a[1] = R.pwlo[b][1];
                pw[b].a[2] = R.pwlo[b][2]; pw[b].a[3] = R.pwlo[b][3]; pw[b].a[4] = R.pwhi[b];
              }
#pragma unroll
              for (int i = 0; i < 5; ++i) own_rt.a[i] = R.r16t[i];
            }
          } else {
            own_len = 0;  // beyond the segment scratch: the generic kernel has it
          }
        }
      }
      own_in_lo = (uint32_t)ioff; own_in_hi = (uint32_t)(ioff >> 32);
      own_out_lo = (uint32_t)ooff; own_out_hi = (uint32_t)(ooff >> 32);
      own_inplace = in + ioff == out + ooff;
      own_nlo = (uint32_t)n;
      own_nhi = (uint32_t)(n >> 32);
      if (MODE == kMTDesc) {
        own_bad = ki >= a.nkeys;
        if (own_bad) ki = 0;
        const u32x4 *kp = reinterpret_cast<const u32x4 *>(a.keys + 32ull * ki);
        const u32x4 ka = __builtin_nontemporal_load(kp), kb = __builtin_nontemporal_load(kp + 1);
        own_k[0] = ka.x; own_k[1] = ka.y; own_k[2] = ka.z; own_k[3] = ka.w;
        own_k[4] = kb.x; own_k[5] = kb.y; own_k[6] = kb.z; own_k[7] = kb.w;
        own_bad = own_bad || (ka.x | ka.y | ka.z | ka.w | kb.x | kb.y | kb.z | kb.w) == 0u;
      } else if (MODE == kMTUniform) {
#pragma unroll
        for (int i = 0; i < 8; ++i) own_k[i] = kuni[i];
      } else if (!(have && own_q < nlong)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) own_k[i] = 0u;
      }
    }
    // the super-tile's body: EX = every record in it is exactly L bytes
    // long (the exact-size records of a descriptor class come first in idx),
    // the body then compiles to the exact-size kernel's -- no masks, no
    // leading absent chunks, no r^(16 - t), whole-piece stores only
    auto run = [&](auto ex_tag) {
    constexpr bool EX = decltype(ex_tag)::value;
    // t = 4 C - P: Poly1305 blocks the record's last ChaCha chunk lacks
    const uint32_t own_t = EX ? 0u : 4u * ((own_len + 63u) >> 6) - ((own_len + 15u) >> 4);

    // the first tile's DMA goes out before the key block and lands meanwhile
    // a record's length and offsets by its key lane kl: computed in the
    // uniform mode (record super0 + kl: no cross-lane traffic), read from the
    // key lane otherwise -- *_s for a wave-uniform kl (v_readlane into SGPRs),
    // *_v for a per-lane kl (ds_bpermute)
    constexpr uint32_t TAGB = TAG_IN ? 31u : 15u;  // input pieces: (len + TAGB) >> 4
    auto len_s = [&](uint32_t kl) -> uint32_t {
      if (EX) return (uint32_t)L;
      return MODE == kMTUniform ? a.len : (uint32_t)__builtin_amdgcn_readlane((int)own_len, (int)kl);
    };
    auto len_v = [&](uint32_t kl) -> uint32_t {
      if (EX) return (uint32_t)L;
      return MODE == kMTUniform ? a.len : (uint32_t)__shfl((int)own_len, (int)kl);
    };
    auto in_s = [&](uint32_t kl) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + kl) * a.in_stride;
      return join64((uint32_t)__builtin_amdgcn_readlane((int)own_in_hi, (int)kl),
                    (uint32_t)__builtin_amdgcn_readlane((int)own_in_lo, (int)kl));
    };
    auto in_v = [&](uint32_t kl) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + kl) * a.in_stride;
      return join64((uint32_t)__shfl((int)own_in_hi, (int)kl), (uint32_t)__shfl((int)own_in_lo, (int)kl));
    };
    auto out_s = [&](uint32_t kl) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + kl) * a.out_stride;
      return join64((uint32_t)__builtin_amdgcn_readlane((int)own_out_hi, (int)kl),
                    (uint32_t)__builtin_amdgcn_readlane((int)own_out_lo, (int)kl));
    };
    auto out_v = [&](uint32_t kl) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + kl) * a.out_stride;
      return join64((uint32_t)__shfl((int)own_out_hi, (int)kl), (uint32_t)__shfl((int)own_out_lo, (int)kl));
    };
    // record klb + sub (sub = 0 .. RPI-1 per lane): SUB_KIB classes
    auto sel_q = [&](uint32_t own, uint32_t klb, uint32_t sub) -> uint32_t {
      uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)own, (int)klb);
#pragma unroll
      for (int k = 1; k < RPI; ++k) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)own, (int)(klb + k));
        v = sub == (uint32_t)k ? w : v;
      }
      return v;
    };
    auto len_q = [&](uint32_t klb, uint32_t sub) -> uint32_t {
      if (EX) return (uint32_t)L;
      return MODE == kMTUniform ? a.len : sel_q(own_len, klb, sub);
    };
    auto in_q = [&](uint32_t klb, uint32_t sub) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + klb + sub) * a.in_stride;
      return join64(sel_q(own_in_hi, klb, sub), sel_q(own_in_lo, klb, sub));
    };
    auto out_q = [&](uint32_t klb, uint32_t sub) -> uint64_t {
      if (MODE == kMTUniform) return (super0 + klb + sub) * a.out_stride;
      return join64(sel_q(own_out_hi, klb, sub), sel_q(own_out_lo, klb, sub));
    };
    auto load_tile = [&](uint64_t rec0, uint32_t t_rpt) {
      const uint64_t left = nrec - rec0;
      const uint32_t nv = left < (uint64_t)RPT ? (uint32_t)left : (uint32_t)RPT;
      constexpr int IN_SLOTS = TAG_IN ? NSLOT : REC_SLOTS;
      if constexpr (WHOLE_KIB) {
        // instruction q: KiB q % KPR of record q / KPR, a wave-uniform base
#pragma unroll
        for (int q = 0; q < REC_SLOTS / 64; ++q) {
          const uint32_t kl = t_rpt + (uint32_t)q / KPR;
          const uint32_t np = (len_s(kl) + TAGB) >> 4;
          const uint32_t kib = 64u * ((uint32_t)q % KPR);
          if ((uint32_t)(q / KPR) < nv && kib < np) {
            const uint64_t off = in_s(kl) + 1024ull * ((uint32_t)q % KPR);
            const uint32_t pc = kib + glq<256>(gl, q);
            if (pc < np) lds_dma16_s(in + off, 16u * glq<256>(gl, q), (lds_void *)(NOISE_LDS3(lds) + 64 * q));
          }
        }
        if (TAG_IN) {  // piece SPR of record r (the tag of a full-size record) -> tag slot r
          const uint32_t r = lane < (uint32_t)RPT ? lane : 0u;
          const uint32_t src = t_rpt + r;
          const uint64_t off = in_v(src);
          const uint32_t np = (len_v(src) + TAGB) >> 4;
          if (lane < (uint32_t)RPT && lane < nv && np > (uint32_t)SPR)
            lds_dma16_v(in + off + 16u * SPR, (lds_void *)(NOISE_LDS3(lds) + REC_SLOTS));
        }
      } else if constexpr (SUB_KIB) {
        // instruction q: records q RPI .. q RPI + RPI-1; slot 64q + lane holds
        // piece swz(64q + lane) = 64q + glq (swz stays inside 16-slot groups)
#pragma unroll
        for (int q = 0; q < REC_SLOTS / 64; ++q) {
          const uint32_t gq = glq<256>(gl, q);
          const uint32_t sub = gq / SPR, p = gq % SPR;
          const uint32_t klb = t_rpt + (uint32_t)q * RPI;
          const uint32_t np = (len_q(klb, sub) + TAGB) >> 4;
          const uint64_t off = in_q(klb, sub);  // every lane reads (the emulator's readlane is collective)
          if ((uint32_t)q * RPI + sub < nv && p < np)
            lds_dma16_v(in + off + 16u * p, (lds_void *)(NOISE_LDS3(lds) + 64 * q));
        }
        if (TAG_IN) {  // as above
          const uint32_t r = lane < (uint32_t)RPT ? lane : 0u;
          const uint32_t src = t_rpt + r;
          const uint64_t off = in_v(src);
          const uint32_t np = (len_v(src) + TAGB) >> 4;
          if (lane < (uint32_t)RPT && lane < nv && np > (uint32_t)SPR)
            lds_dma16_v(in + off + 16u * SPR, (lds_void *)(NOISE_LDS3(lds) + REC_SLOTS));
        }
      } else {
        // one DMA per iteration (as tile_kernel.hpp's): unrolled, every
        // piece's shuffled address is live at once and the classes below
        // 1 KiB spill
#pragma unroll 1
        for (int q = 0; q < (IN_SLOTS + 63) / 64; ++q) {
          const uint32_t s = 64u * q + lane;
          uint32_t r, p;
          if (s < (uint32_t)REC_SLOTS) {
            const uint32_t g = mpiece<S>(s);
            r = g / SPR;
            p = g % SPR;
          } else {  // tag slots
            r = s - REC_SLOTS;
            p = SPR;
          }
          const uint32_t src = t_rpt + (r < (uint32_t)RPT ? r : 0u);
          const uint64_t off = in_v(src);
          const uint32_t np = (len_v(src) + TAGB) >> 4;
          if (s < (uint32_t)IN_SLOTS && r < nv && p < np)
            lds_dma16_v(in + off + 16u * p, (lds_void *)(NOISE_LDS3(lds) + 64 * q));
        }
      }
    };
    load_tile(super0, 0u);

    if (!TAIL) {  // ChaCha block 0: r, s; G > 1: r^BPL, r^(2 BPL), ...
      uint32_t otk[16];
      chacha20_block(own_k, 0u, own_nlo, own_nhi, otk);
      kr[0] = otk[0] & 0x0fffffffu;
      kr[1] = otk[1] & 0x0ffffffcu;
      kr[2] = otk[2] & 0x0ffffffcu;
      kr[3] = otk[3] & 0x0ffffffcu;
      kss[0] = otk[4]; kss[1] = otk[5]; kss[2] = otk[6]; kss[3] = otk[7];
      if (G > 1) {
        static_assert(G == 1 || BPL == 16, "lanes of 16 Poly1305 blocks");
        F26 x = to26(kr[0], kr[1], kr[2], kr[3], 0u);
        const F26 x1 = x;
        const F26 x2 = mul26(x1, x1), x4 = mul26(x2, x2), x8 = mul26(x4, x4);
        x = mul26(x8, x8);
        pw[0] = x;
        // r^(16 - t): the weight of a full lane's sum past the lane before
        // the record's last (module comment); t = 4 C - P blocks short
        const uint32_t tt = own_t;
        if (!EX && __ballot(tt != 0u)) {
          const F26 one = to26(1u, 0u, 0u, 0u, 0u);
          F26 y = mul26(x8, x4);                                // r^12
          y = mul26(y, (tt == 1u || tt == 2u) ? x2 : one);      // r^14 (t <= 2)
          own_rt = mul26(y, (tt == 1u || tt == 3u) ? x1 : one); // r^15 (t = 1), r^13 (t = 3)
          if (tt == 0u) own_rt = x;
        }
#pragma unroll
        for (int b = 1; b < C::LOG2G; ++b) pw[b] = mul26(pw[b - 1], pw[b - 1]);
      }
    }

#pragma unroll 1
    for (int t = 0; t < NTS; ++t) {
      const uint64_t rec0 = super0 + (uint64_t)t * RPT;
      if (rec0 >= nrec) break;
      const uint32_t nv = (nrec - rec0) < (uint64_t)RPT ? (uint32_t)(nrec - rec0) : (uint32_t)RPT;
      wait_vmem();
      wave_lds_fence();
      const uint32_t src = (uint32_t)t * RPT + rho;  // key lane of my record
      const bool valid = !idle && rho < nv;
      // ---- this lane's record ------------------------------------------
      const uint32_t rlen = len_v(src);
      const uint32_t P = (rlen + 15u) >> 4, Cc = (rlen + 63u) >> 6;
      const uint32_t F = rlen >> 4, sb = rlen & 15u;  // whole pieces, bytes in the last one
      const int dc = (int)(L / 64) - (int)Cc;  // leading absent chunks
      const uint32_t rbase = rho * SPR;
      auto pslot = [&](uint32_t i) -> uint32_t {  // record piece i (0 .. SPR) -> slot
        return i < (uint32_t)SPR ? mslot<S>(rbase + i) : (uint32_t)REC_SLOTS + rho;
      };
      Poly1305 p;
      p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
      p.r0 = p.r1 = p.r2 = p.r3 = 0u;
      p.s0 = p.s1 = p.s2 = p.s3 = 0u;
      if (DO_POLY) {
        p.r0 = __shfl(kr[0], src); p.r1 = __shfl(kr[1], src);
        p.r2 = __shfl(kr[2], src); p.r3 = __shfl(kr[3], src);
        p.s0 = __shfl(kss[0], src); p.s1 = __shfl(kss[1], src);
        p.s2 = __shfl(kss[2], src); p.s3 = __shfl(kss[3], src);
      }
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      uint32_t kt[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) kt[i] = DO_XOR ? (KEYED ? (uint32_t)__shfl((int)own_k[i], (int)src) : kuni[i]) : 0u;
      uint32_t n_lo = 0u, n_hi = 0u, cbase = 1u;
      if (DO_XOR) {
        if (KEYED) {
          n_lo = (uint32_t)__shfl((int)own_nlo, (int)src);
          n_hi = (uint32_t)__shfl((int)own_nhi, (int)src);
        } else {
          const uint64_t n = a.nonce0 + rec0 + rho;
          n_lo = (uint32_t)n;
          n_hi = (uint32_t)(n >> 32);
        }
        if (TAIL) cbase += (uint32_t)__shfl((int)own_cb, (int)src);
      }
      const bool bad_key = MODE == kMTDesc && __shfl((int)own_bad, (int)src) != 0;

      // ---- decrypt: the tag out of the tile (bytes rlen .. rlen + 15) ------
      uint4 want = make_uint4(0u, 0u, 0u, 0u);
      if (TAG_IN) {
        const uint4 A = lb[pslot(F)];
        const uint4 B = lb[sb ? pslot(F + 1u) : (uint32_t)ZSLOT];
        want = sb ? extract16(A, B, sb) : A;
      }
      wave_lds_fence();  // the tag is read before lane G-1's XOR rewrites its first piece

      // ---- ChaCha20 XOR and Poly1305, right-aligned by whole chunks ------
      // (the top of the file).  As in tile_kernel.hpp, ONE LDS read of a
      // piece feeds both the XOR and the MAC, and the ChaCha block of chunk
      // kk + 1 is computed beside the XOR / MAC of chunk kk.  Leading absent
      // chunks: garbage in a junk slot, h reset to 0 after each of them.  The
      // last chunk (lane G-1's, the record's last real one): the MAC input is
      // masked to the record's bytes (zero padding), and its trailing absent
      // blocks (past P) multiply by r = 1 with no 2^128 bit -- identities.
      const int rc0 = (int)(CPL * j) - dc;  // real chunk of my virtual chunk 0
      const uint32_t lbytes = j == (uint32_t)G - 1u ? rlen - 64u * (Cc - 1u) : 64u;  // bytes in my last chunk
      const uint32_t lblk = (lbytes + 15u) >> 4;                                      // blocks in it (1..4)
      ChaPre pre{};
      if (DO_XOR) pre = chacha_pre(kt, n_lo, n_hi);
      uint32_t ks[16];
      if (DO_XOR) chacha20_block_pre(kt, cbase + (uint32_t)rc0, pre, n_lo, n_hi, ks);
#pragma unroll
      for (int kk = 0; kk < CPL; ++kk) {
        const int c = rc0 + kk;
        uint32_t ksn[16];
        if (DO_XOR && kk + 1 < CPL) chacha20_block_pre(kt, cbase + (uint32_t)(c + 1), pre, n_lo, n_hi, ksn);
        const bool last = kk == CPL - 1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t slot = (EX || c >= 0) && !idle ? mslot<S>(rbase + 4u * (uint32_t)c + (uint32_t)q) : (uint32_t)JSLOT;
          const uint4 v = lb[slot];
          uint4 o = v;
          if (DO_XOR) {
            o.x = v.x ^ ks[4 * q + 0];
            o.y = v.y ^ ks[4 * q + 1];
            o.z = v.z ^ ks[4 * q + 2];
            o.w = v.w ^ ks[4 * q + 3];
            lb[slot] = o;
          }
          if (DO_POLY) {
            uint4 m = POLY_PRE ? v : o;
            if (!EX && last) {
              // the record's last chunk: bytes past rlen (tag bytes, stale
              // pieces, keystream) must not reach the MAC
              const int nb = (int)lbytes - 16 * q;
              const uint4 mk = mtab[nb <= 0 ? 0 : (nb >= 16 ? 16 : nb)];
              m.x &= mk.x; m.y &= mk.y; m.z &= mk.z; m.w &= mk.w;
            }
            if (!EX && last && q > 0) {  // a trailing absent block is the identity (r = 1, no 2^128)
              const bool on = (uint32_t)q < lblk;
              poly_block_r(p, m.x, m.y, m.z, m.w, on ? 1u : 0u, on ? p.r0 : 1u, on ? p.r1 : 0u,
                           on ? p.r2 : 0u, on ? p.r3 : 0u, on ? p.rr0 : 0u, on ? p.rr1 : 0u,
                           on ? p.rr2 : 0u, on ? p.rr3 : 0u, on ? p.r0lo : 1u);
            } else {
              poly_block(p, m.x, m.y, m.z, m.w);
            }
          }
        }
        if (DO_POLY && !EX && c < 0) {  // a leading absent chunk: start the Horner chain over
          p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
        }
        if (DO_XOR && kk + 1 < CPL) {
#pragma unroll
          for (int i = 0; i < 16; ++i) ks[i] = ksn[i];
        }
      }

      // ---- recombination: sum_j acc_j r^(BPL (G-1-j)) (tile_kernel.hpp) --
      if (DO_POLY && G > 1) {
        // lane j's sum is followed by BPL (G-1-j) - t real blocks: weight
        // r^(BPL (G-2-j)) r^(16 - t) for j < G-1, 1 for the last lane (t = 0
        // in the whole tile: the exact-size weights r^(BPL (G-1-j)))
        F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
        const uint32_t rt_t = 4u * Cc - P;
        const bool any_t = !EX && __ballot(valid && rt_t != 0u) != 0;
        const uint32_t m = any_t ? (j + 1u < (uint32_t)G ? (uint32_t)G - 2u - j : 0u) : (uint32_t)G - 1u - j;
#pragma unroll
        for (int b = 0; b < C::LOG2G; ++b) {
          F26 f;
          const bool use = (m >> b) & 1u;
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const uint32_t w = __shfl(pw[b].a[i], src);
            f.a[i] = use ? w : (i == 0 ? 1u : 0u);
          }
          h = mul26(h, f);
        }
        if (any_t) {  // wave-uniform
          F26 f;
          const bool use = j + 1u < (uint32_t)G;
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const uint32_t w = __shfl(own_rt.a[i], src);
            f.a[i] = use ? w : (i == 0 ? 1u : 0u);
          }
          h = mul26(h, f);
        }
        if constexpr ((G & (G - 1)) == 0) {  // butterfly: every lane of the record gets the sum
#pragma unroll
          for (int b = 0; b < C::LOG2G; ++b) {
            if (b == 4) carry26(h);
#pragma unroll
            for (int i = 0; i < 5; ++i) h.a[i] += __shfl_xor(h.a[i], 1 << b);
          }
        } else {  // G lanes not a power of two: a tree into lane j = 0 (the only user)
#pragma unroll
          for (int b = 0; b < C::LOG2G; ++b) {
            if (b == 4) carry26(h);
            const bool in = j + (1u << b) < (uint32_t)G;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
              const uint32_t w = (uint32_t)__shfl((int)h.a[i], (int)((lane + (1u << b)) & 63u));
              h.a[i] += in ? w : 0u;
            }
          }
        }
        carry26(h);
        carry26(h);
        from26(h, p.h0, p.h1, p.h2, p.h3, p.h4);
      }
      uint32_t tag[4] = {0u, 0u, 0u, 0u};
      if (!TAIL) {
        poly_block(p, 0u, 0u, rlen, 0u);  // LE64(ad_len = 0) || LE64(len)
        poly_final(p, tag);
      }

      // ---- outcome per record --------------------------------------------
      uint64_t fail_mask = 0;  // bit r * G: record r of this tile is not output as computed
      const uint64_t badk_mask = __ballot(j == 0 && bad_key);
      fail_mask = badk_mask;
      const uint32_t rec_di = MODE == kMTDesc ? (uint32_t)__shfl((int)own_di, (int)src) : 0u;
      const bool rec_inplace = __shfl((int)own_inplace, (int)src) != 0;
      const uint64_t inpl_mask = __ballot(j == 0 && rec_inplace);
      if (TAG_IN) {
        const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) | (want.w ^ tag[3]);
        fail_mask |= __ballot(j == 0 && valid && diff != 0u);
        if (j == 0 && valid) {
          const uint64_t si = MODE == kMTDesc ? (uint64_t)rec_di : rec0 + rho;
          a.status[si] = bad_key ? 2u : (diff ? 1u : 0u);
        }
      } else if (MODE == kMTTailXor) {  // the record's tag failed: its tail is not output
        const bool rec_ok = __shfl((int)own_ok, (int)src) != 0;  // every lane shuffles
        fail_mask |= __ballot(j == 0 && valid && !rec_ok);
      }
      {
        // P_tail -> the SegRec, for k_seg_finalize_w (shuffle outside divergent code)
        const uint32_t q = TAIL ? (uint32_t)__shfl((int)own_q, (int)src) : 0u;
        if (TAIL && DO_POLY && j == 0 && valid && rlen != 0u) {  // rlen 0: past the scratch
          SegRec &R = const_cast<SegRec &>(a.rt[q]);
          R.ptail[0] = p.h0; R.ptail[1] = p.h1; R.ptail[2] = p.h2; R.ptail[3] = p.h3;
          R.ptail[4] = p.h4;
        }
      }
      if (TAG_OUT && j == 0 && valid) {  // the tag at byte rlen of the output image
        const uint4 T = make_uint4(tag[0], tag[1], tag[2], tag[3]);
        if (sb == 0u) {
          lb[pslot(F)] = T;
        } else {
          const uint4 Z = make_uint4(0u, 0u, 0u, 0u);
          const uint4 A = mask_bytes(lb[pslot(F)], (int)sb);  // ciphertext bytes before rlen
          const uint4 lo = extract16(Z, T, 16u - sb), hi = extract16(T, Z, 16u - sb);
          lb[pslot(F)] = make_uint4(A.x | lo.x, A.y | lo.y, A.z | lo.z, A.w | lo.w);
          lb[pslot(F + 1u)] = hi;
        }
      }
      wave_lds_fence();
      if (!DO_XOR) {  // tail Poly1305 pass: nothing to store; the next tile's DMA
        if (t + 1 < NTS && rec0 + RPT < nrec) {
          wait_lds();
          wave_lds_fence();
          load_tile(rec0 + RPT, (uint32_t)(t + 1) * RPT);
        }
        continue;
      }

      // ---- gather the outputs, next tile's DMA, stores ------------------
      // output bytes of record r: len + 16 (encrypt with tag) or len.  The
      // whole pieces go out as 16-byte stores, in NPART parts (fewer pieces
      // live in registers); the next tile's DMA overwrites the tile, so it
      // is issued after the last part's gather, before that part's stores.
      // Only the gathered pieces live across the DMA: each store's record,
      // guard and address are worked out after it.
      constexpr bool REG = WHOLE_KIB || SUB_KIB;  // record pieces, then one instruction of tags
      constexpr int NOUT = REG ? (REC_SLOTS / 64 + (TAG_OUT ? 1 : 0)) : (RPT * OPR + 63) / 64;
      // (per-lane records below 1 KiB: every store shuffles its record's
      // length and offset, so parts of <= 6 pieces -- more spill)
      constexpr int NPART = REG ? (NOUT > 8 ? 2 : 1) : (NOUT + 5) / 6;
      constexpr int NQ = (NOUT + NPART - 1) / NPART;
      const bool full = nv == (uint32_t)RPT;
      // output piece q of this lane: its record r, piece index pc, tile slot
      auto piece = [&](int q, uint32_t &r, uint32_t &pc, uint32_t &slot, bool &ok) {
        if (WHOLE_KIB && q < REC_SLOTS / 64) {  // KiB q % KPR of record q / KPR
          r = (uint32_t)q / KPR;
          pc = 64u * ((uint32_t)q % KPR) + lane;
          slot = swz<256>(64u * q + lane);
          ok = true;
        } else if (SUB_KIB && q < REC_SLOTS / 64) {  // records q RPI + lane / SPR
          r = (uint32_t)q * RPI + lane / SPR;
          pc = lane % SPR;
          slot = swz<256>(64u * q + lane);
          ok = true;
        } else if (REG) {  // the tag slots (piece SPR), lane r -> record r
          r = lane < (uint32_t)RPT ? lane : 0u;
          pc = SPR;
          slot = REC_SLOTS + r;
          ok = lane < (uint32_t)RPT;
        } else {
          const uint32_t g = 64u * q + lane;
          r = g / OPR;
          pc = g % OPR;
          ok = (RPT * OPR) % 64 == 0 || g < (uint32_t)(RPT * OPR);
          if (!ok) r = 0;
          slot = pc < (uint32_t)SPR ? mslot<S>(r * SPR + pc) : (uint32_t)REC_SLOTS + r;
        }
      };
      const uint32_t pr = lane < (uint32_t)RPT ? lane : 0u;  // the partial piece's record
#pragma unroll
      for (int part = 0; part < NPART; ++part) {
        uint4 ov[NQ];
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const int q = part * NQ + qq;
          ov[qq] = make_uint4(0u, 0u, 0u, 0u);
          if (q >= NOUT) break;
          uint32_t r, pc, slot;
          bool ok;
          piece(q, r, pc, slot, ok);
          ov[qq] = lb[slot];
        }
        // the partial last piece of record `lane` (read before the DMA)
        uint4 pv = make_uint4(0u, 0u, 0u, 0u);
        if (part == NPART - 1) {
          if (!EX) {
            const uint32_t ob = len_v((uint32_t)t * RPT + pr) + (TAG_OUT ? 16u : 0u);
            const uint32_t pp = ob >> 4;  // its piece index
            const uint32_t slot = pp < (uint32_t)SPR ? mslot<S>(pr * SPR + pp) : (uint32_t)REC_SLOTS + pr;
            pv = lb[(ob & 15u) ? slot : (uint32_t)ZSLOT];
          }
          wait_lds();  // every LDS read of this tile done
          wave_lds_fence();
          if (t + 1 < NTS && rec0 + RPT < nrec) load_tile(rec0 + RPT, (uint32_t)(t + 1) * RPT);
        }
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const int q = part * NQ + qq;
          if (q >= NOUT) break;
          uint32_t r, pc, slot;
          bool ok;
          piece(q, r, pc, slot, ok);
          const uint32_t kl = (uint32_t)t * RPT + r;
          uint32_t ln;
          uint64_t ob;
          if (WHOLE_KIB && q < REC_SLOTS / 64) {  // one record per instruction: wave-uniform
            ln = len_s(kl);
            ob = out_s(kl);
          } else if (SUB_KIB && q < REC_SLOTS / 64) {
            const uint32_t klb = (uint32_t)t * RPT + (uint32_t)q * RPI;
            ln = len_q(klb, lane / SPR);
            ob = out_q(klb, lane / SPR);
          } else {
            ln = len_v(kl);
            ob = out_v(kl);
          }
          const uint32_t nfo = (ln + (TAG_OUT ? 16u : 0u)) >> 4;  // whole output pieces
          bool st = ok && (full || r < nv) && pc < nfo;
          uint4 v = ov[qq];
          if ((fail_mask >> (r * G)) & 1u) {  // not output as computed (rare)
            const bool bk = ((badk_mask >> (r * G)) & 1u) != 0;
            const bool inpl = ((inpl_mask >> (r * G)) & 1u) != 0;
            st = st && DECRYPT && !inpl && !bk;
            v = make_uint4(0u, 0u, 0u, 0u);
          }
          if (st) store16<true>(out + ob + 16ull * pc, v, 16);
        }
        if (!EX && part == NPART - 1) {
          const uint32_t kl = (uint32_t)t * RPT + pr;
          const uint32_t ob = len_v(kl) + (TAG_OUT ? 16u : 0u);
          const uint64_t obase = out_v(kl);
          uint32_t pn = ob & 15u;
          if (!(lane < (uint32_t)RPT && lane < nv)) pn = 0u;
          if ((fail_mask >> (pr * G)) & 1u) {
            const bool bk = ((badk_mask >> (pr * G)) & 1u) != 0;
            const bool inpl = ((inpl_mask >> (pr * G)) & 1u) != 0;
            if (!DECRYPT || inpl || bk) pn = 0u;
            pv = make_uint4(0u, 0u, 0u, 0u);
          }
          if (pn) store_head(out + obase + 16ull * (ob >> 4), pv, pn);
        }
      }
    }
    };  // run
    bool ex = false;
    if (MODE == kMTDesc)
      ex = __ballot(lane < (uint32_t)RPS && super0 + lane < nrec && own_len != (uint32_t)L) == 0;
    if constexpr (MODE == kMTDesc) {
      if (ex)
        run(std::true_type{});
      else
        run(std::false_type{});
    } else {
      run(std::false_type{});
    }
  }
}

}  // namespace noise_amd
