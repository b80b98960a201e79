// tile_kernel.hpp -- the LDS-staged ("tile") AEAD kernel for uniform-length,
// 16-byte aligned, AD-free record batches (the transport hot path).
//
// Why: the lane-per-record walk reads/writes each record in 16-byte pieces
// spread over 64 records per wave-instruction; on MI355X that access shape
// runs at ~0.5 TB/s.  Whole-record, lane-contiguous wave-instructions (1 KiB
// each) run at copy speed.  So records move HBM <-> LDS in whole-record,
// coalesced wave-instructions (LDS-DMA `global_load_lds_dwordx4` in,
// `ds_read_b128` + `global_store_dwordx4` out) and the arithmetic reads its
// pieces from LDS.
//
// Work split (one 64-thread workgroup = one wave = one "super-tile" of 64
// consecutive records):
//   * key pass: lane l computes ChaCha block 0 of record l (r, s) and, for
//     G > 1, the Poly1305 powers r^16, r^32, ... it will hand out;
//   * G = max(1, L/256) lanes per record, RPT = 64/G records per tile,
//     G tiles per super-tile.  Lane j of a record owns the contiguous
//     256-byte span [256j, 256j+256): 4 ChaCha blocks (counters 1+4j..4+4j)
//     and 16 Poly1305 blocks, Horner-evaluated with the clamped r;
//   * the G partial sums recombine as  sum_j acc_j * r^(16(G-1-j)),
//     log2(G) general products per lane + a log2(G)-step butterfly.
// Per tile the wave does: compute (LDS in place) -> gather the output
// records into VGPRs -> issue the NEXT tile's LDS-DMA and THIS tile's global
// stores back to back, so the two memory round trips overlap; the only
// memory wait is the one before the next compute.  A workgroup is a single
// wave, so no s_barrier is needed: LDS ordering is program order within the
// wave (the fences below only stop the compiler from moving LDS accesses).
// LDS image per tile: RPT*L/16 16-byte slots (plaintext/ciphertext, XOR-
// swizzled (swz) so the per-lane ds_read/ds_write_b128 are bank-conflict
// free) + RPT tag slots.  The swizzle is applied on the
// global SOURCE address of the LDS-DMA (its LDS destination is lane-linear).
#pragma once
#include "chachapoly_device.hpp"

namespace noise_amd {

// SPAN: bytes of a record per lane (256: 4 ChaCha blocks / 16 Poly1305
// blocks per lane; 128 halves the tile: twice the lanes per record)
template <int L, int SPAN = 256>
struct TileCfg {
  static constexpr int G = L >= SPAN ? L / SPAN : 1;  // lanes per record
  static constexpr int RPT = 64 / G;                // records per tile
  static constexpr int CPL = (L / 64) / G;          // 64-B chunks per lane
  static constexpr int BPL = 4 * CPL;               // Poly1305 blocks per lane
  static constexpr int SPR = L / 16;                // 16-B slots per record
  static constexpr int REC_SLOTS = RPT * SPR;
  static constexpr int NSLOT = REC_SLOTS + RPT;     // + one tag slot per record
  static constexpr int LOG2G = G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3
                              : G == 16 ? 4 : G == 32 ? 5 : 6;
  static constexpr int LOG2BPL = BPL == 4 ? 2 : BPL == 8 ? 3 : BPL == 16 ? 4 : 5;
  static_assert(L % 64 == 0 && 64 % G == 0 && (L < SPAN || L % SPAN == 0), "tile shape");
  static_assert(G == 1 || BPL == 8 || BPL == 16, "span of 128 or 256 bytes");
};

// slot <-> piece involution (gfx950 banking: ds_read_b128 in four 16-lane
// groups over 16 slots of 16 B, ds_write_b128 in eight 8-lane groups over 8).
// SPAN 256 (lanes 4 apart share a record): XOR within each aligned 16-slot
// group by slot bits 4..7 -- lane l's span starts at slot 16l.  SPAN 128
// (lane l's span at slot 8l): XOR of bits 0..2 by bits 3..5 ^ 6..8, which
// keeps the 8-lane write groups conflict free as well (the 256-B form leaves
// lanes 2k, 2k+1 on one bank of a ds_write_b128: 2-way, 8.7 M extra LDS
// cycles per keystream-pass launch in config 4).
template <int SPAN>
__device__ __forceinline__ uint32_t swz(uint32_t s) {
  if constexpr (SPAN == 128) return s ^ (((s >> 3) ^ (s >> 6)) & 7u);
  else return s ^ ((s >> 4) & 15u);
}
// swz(64q + lane) - 64q from gl[i] = swz(64i + lane) - 64i: it depends on q
// only through q & 3 (SPAN 256), or is gl[0] ^ (q & 7) (SPAN 128)
template <int SPAN>
__device__ __forceinline__ uint32_t glq(const uint32_t gl[4], int q) {
  if constexpr (SPAN == 128) return gl[0] ^ ((uint32_t)q & 7u);
  else return gl[q & 3];
}

// LDS-typed pointer for the LDS-DMA destinations.  Taking it straight from
// the __shared__ array (instead of casting a generic pointer inside a
// helper) keeps the address space static: a generic->LDS cast that the
// compiler cannot fold makes ROCm 7.2's gfx950 backend emit an illegal
// V_CMP on src_shared_base when many kernels share one module.
typedef __attribute__((address_space(3))) uint4 lds_u4;
#define NOISE_LDS3(arr) ((lds_u4 *)(arr))

// compiler-level LDS ordering point for a single-wave workgroup
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Record addressing / keying of a tile launch.
enum TileMode : int {
  kTileUniform = 0,   // one key, nonce0 + i, record i at in + i*in_stride
  kTileSessions = 1,  // key row keys[key_idx[i]], nonce nonces[i], strided
  // 2: round 5's descriptor classes, now k_aead_mtile's kMTDesc
  kTileSeg = 3,       // 1 KiB segment g of a long record (segs[g] -> SegRec):
                      // ciphertext + Poly1305 partial sum, no tag (encrypt)
  kTileSegPoly = 4,   // decrypt pass 1: the segment's Poly1305 partial sum of
                      // the ciphertext only (no keystream, nothing stored)
  kTileSegXor = 5,    // decrypt pass 3 (after the tags are checked): keystream
                      // XOR of the segments of VERIFIED records -> plaintext;
                      // a failed record's segment: nothing (in place) / zeros
};

// ---- long records as 1 KiB segments (records_kernels.hip) -----------------
// A record of len >= 1024 bytes is cut into nfull = len / 1024 full segments
// plus a tail of len % 1024 bytes.  Segment s covers bytes [1024 s, 1024 s +
// 1024): ChaCha blocks 1 + 16 s .. 16 + 16 s and Poly1305 blocks 64 s ..
// 64 s + 63.  The tile kernel (kTileSeg) encrypts/decrypts every full
// segment of every long record as if it were a 1 KiB record -- one uniform,
// load-balanced launch -- and leaves the segment's Poly1305 Horner sum
//   P_s = sum_{i<64} m_{64s+i} r^(64-i)
// in SegPartial.  The finalize kernel combines h = sum_s P_s r^(64(nfull-1-s))
// (Horner in R = r^64), appends the tail (the len % 1024 bytes past the last
// full segment, masked 1 KiB tile units of k_aead_mtile) as h r^(tail blocks)
// + P_tail, then the length block and the tag.
struct SegRec {                  // one per long record, 256 B (two 128-B lines)
  uint64_t in_off, out_off, nonce, seg0;  // seg0: index of segment 0
  uint32_t k[8];                 // the record's key (copied from the key table)
  uint32_t key_idx, di, len, nfull;       // di: descriptor index
  uint32_t r[4];                 // clamped Poly1305 r (radix 2^32)
  uint32_t s[4];                 // Poly1305 s
  // r^16, r^32, r^48 (radix 2^26; limbs 0..3 | limb 4): lane j of a
  // segment's four 256-B spans scales its Horner sum by r^(16 (3 - j)) with
  // ONE product from its own load (the tile kernel's kTileSeg* modes)
  uint32_t pwlo[3][4], pwhi[3];
  uint32_t r64[5];               // r^64 (radix 2^26)
  uint32_t rtail[5];             // r^(tail blocks) (radix 2^26)
  uint32_t ptail[5];             // the tail's Poly1305 sum (radix 2^32, h4 small)
  uint32_t ok;                   // decrypt: 1 once the finalize kernel verified the tag
  uint32_t r16t[5];              // r^(16 - t) of the tail's masked tile unit (radix 2^26;
                                 // t = 4 ceil(tail / 64) - ceil(tail / 16), mtile_kernel.hpp)
};
static_assert(sizeof(SegRec) == 256, "SegRec layout");
struct SegEntry {                // one per full segment
  uint32_t q, s;                 // long-record index, segment number
};
struct SegPartial {              // P_s in radix 2^32: words h0..h3 (h4, small,
  uint32_t h[4];                 // in a separate array: 20 B per segment)
};

struct TileArgs {
  KeyArg key;         // kTileUniform
  uint64_t nonce0;    // kTileUniform
  const uint8_t *in;
  uint64_t in_stride;  // kTileUniform / kTileSessions
  uint8_t *out;
  uint64_t out_stride;
  uint8_t *status;    // decrypt: per record (kMTDesc: per descriptor)
  uint64_t nrec;      // kTileUniform / kTileSessions
  int in_place;       // kTileUniform / kTileSessions
  uint32_t nkeys;     // kTileSessions / kMTDesc
  const uint8_t *keys;
  const uint32_t *key_idx;  // kTileSessions
  const uint64_t *nonces;   // kTileSessions
  const noise_gpu_record *recs;  // kMTDesc (mtile_kernel.hpp)
  const uint32_t *idx;           // kMTDesc: class-sorted descriptor indices
  const unsigned long long *cls_base;  // kMTDesc: class start in idx (device)
  const unsigned long long *counts;    // kMTDesc: per-class counts (device)
  int cls;                       // kMTDesc: this launch's class
  int cls2;                      // kMTDesc: the ragged class stored right after cls in idx, or -1
  const SegEntry *segs;         // kTileSeg
  const SegRec *rt;              // kTileSeg
  const unsigned long long *seg_split;  // kTileSeg*: chunk boundaries (device), or null
  int chunk;                     // kTileSeg*: this launch's chunk of seg_split
  SegPartial *partial;           // kTileSeg: P_s words 0..3
  uint32_t *partial_hi;          // kTileSeg: P_s word 4
  const unsigned long long *nseg;  // kTileSeg: number of segments (device)
  // the masked kernel (mtile_kernel.hpp)
  uint32_t len;                         // kMTUniform: every record's length
  const uint32_t *tails;                // kMTTail*: long records with a tail (SegRec index)
  const unsigned long long *ntails;     // kMTTail*: their count (device)
  const unsigned long long *tail_split; // kMTTail*: chunk boundaries in tails (device), or null
  const unsigned long long *nlong;      // kMTTail*: long records in the scratch (device)
};

// kTileSeg*: all segments, or chunk a.chunk of them
__device__ __forceinline__ void seg_range(const TileArgs &a, uint64_t &base, uint64_t &n) {
  base = 0;
  n = *a.nseg;
  if (a.seg_split) {  // chunk c: [split[c], split[c + 1]), clamped to the segments there are
    const uint64_t lo = a.seg_split[a.chunk], hi = a.seg_split[a.chunk + 1];
    base = lo < n ? lo : n;
    n = (hi < n ? hi : n) - base;
  }
}

template <int L, bool DECRYPT, bool CONTIG, int MODE, int ABL, int SPAN>
__device__ __forceinline__ void tile_load(lds_u4 *lds3, const uint8_t *in,
                                          uint64_t in_stride, uint64_t rec0,
                                          uint32_t nv, uint32_t lane,
                                          const uint32_t gl[4],
                                          uint32_t t_rpt, uint32_t own_in_lo,
                                          uint32_t own_in_hi) {
  using C = TileCfg<L, SPAN>;
  if (ABL == 1) return;
  constexpr bool TAGGED_IN = DECRYPT && MODE < kTileSeg;  // ct || tag pieces
  // every record byte is read once: the streaming (nt) policy (lds_dma16_*)
  constexpr int IN_SLOTS = TAGGED_IN ? C::NSLOT : C::REC_SLOTS;
  if (CONTIG) {
    // slot s = 64q + lane holds piece swz(s) = 64q + glq(gl, q); packed
    // records put piece g of an encrypt tile at byte 16g and of a decrypt
    // tile (SPR+1 pieces per record) at 16(g + g/SPR).
    const uint8_t *base = in + rec0 * in_stride;  // wave-uniform
    if (nv >= (uint32_t)C::RPT) {
      // full tile (every tile but a batch's last): no per-instruction guard,
      // which the compiler otherwise turns into a compare, an exec mask and
      // two taken branches around each of the REC_SLOTS / 64 DMAs
#pragma unroll
      for (int q = 0; q < C::REC_SLOTS / 64; ++q) {
        const uint32_t g = 64u * q + glq<SPAN>(gl, q);
        const uint32_t rr = g / C::SPR;
        lds_dma16_s(base, DECRYPT ? 16u * (g + rr) : 16u * g, (lds_void *)(lds3 + 64 * q));
      }
    } else {
#pragma unroll
      for (int q = 0; q < C::REC_SLOTS / 64; ++q) {
        const uint32_t g = 64u * q + glq<SPAN>(gl, q);
        const uint32_t rr = g / C::SPR;
        const uint32_t off = DECRYPT ? 16u * (g + rr) : 16u * g;
        if (rr < nv) lds_dma16_s(base, off, (lds_void *)(lds3 + 64 * q));
      }
    }
    if (TAGGED_IN) {  // tag pieces: slot REC_SLOTS + r <- piece (r, SPR)
#pragma unroll
      for (int q = C::REC_SLOTS / 64; q < (C::NSLOT + 63) / 64; ++q) {
        const uint32_t r = 64u * q + lane - C::REC_SLOTS;
        if (r < nv)
          lds_dma16_s(base, 16u * (r * (C::SPR + 1) + C::SPR), (lds_void *)(lds3 + 64 * q));
      }
    }
  } else if (MODE >= kTileSeg) {
    // whole KiB (segments): DMA
    // instruction q moves KiB q % (SPR / 64) of unit q / (SPR / 64), so its
    // offset is wave-uniform -- read from the unit's key lane (v_readlane into
    // SGPRs) instead of a per-lane shuffle
    constexpr int KPR = C::SPR / 64;  // KiB per unit
#pragma unroll
    for (int q = 0; q < C::REC_SLOTS / 64; ++q) {
      if ((uint32_t)(q / KPR) < nv) {
        const uint32_t kl = t_rpt + q / KPR;
        const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)own_in_hi, (int)kl),
                                    (uint32_t)__builtin_amdgcn_readlane((int)own_in_lo, (int)kl)) +
                             1024ull * (q % KPR);
        lds_dma16_s(in + off, 16u * glq<SPAN>(gl, q), (lds_void *)(lds3 + 64 * q));
      }
    }
    if (TAGGED_IN) {  // decrypt: the RPT tags, lane r -> slot REC_SLOTS + r
      const uint32_t r = lane < (uint32_t)C::RPT ? lane : 0u;
      const uint64_t off = ((uint64_t)(uint32_t)__shfl((int)own_in_hi, (int)(t_rpt + r)) << 32) |
                           (uint32_t)__shfl((int)own_in_lo, (int)(t_rpt + r));
      if (lane < (uint32_t)C::RPT && lane < nv)
        lds_dma16_v(in + off + 16u * C::SPR, (lds_void *)(lds3 + C::REC_SLOTS));
    }
  } else {
#pragma unroll 1
    for (int q = 0; q < (IN_SLOTS + 63) / 64; ++q) {
      const uint32_t s = 64u * q + lane;
      uint32_t r, p;
      if (s < (uint32_t)C::REC_SLOTS) {
        const uint32_t g = swz<SPAN>(s);
        r = g / C::SPR;
        p = g % C::SPR;
      } else {  // decrypt: tag slots
        r = s - C::REC_SLOTS;
        p = C::SPR;
      }
      const uint8_t *rec_base;
      if (MODE >= kTileSeg) {  // offset of record r: key lane t*RPT + r
        const uint32_t src = t_rpt + (r < (uint32_t)C::RPT ? r : 0u);
        const uint64_t off = ((uint64_t)(uint32_t)__shfl((int)own_in_hi, src) << 32) |
                             (uint32_t)__shfl((int)own_in_lo, src);
        rec_base = in + off;
      } else {
        rec_base = in + (rec0 + r) * in_stride;
      }
      if (s < (uint32_t)IN_SLOTS && r < nv)
        lds_dma16_v(rec_base + 16u * p, (lds_void *)(lds3 + 64 * q));
    }
  }
}

// MODE kTileSessions: record i uses key row keys[key_idx] and its own
// nonce; a key index outside the table makes the record fail (nothing
// written; decrypt status NOISE_GPU_REC_BAD_KEY).
// kTileSeg (L = 1024): unit i is full segment i of a long record (SegEntry ->
// SegRec): no key block (r and its powers come from the SegRec), ChaCha
// counters 1 + 16 s + ..., no tag: the segment's Poly1305 partial sum goes to
// a.partial[i] (encrypt).  Decrypt splits the same unit into kTileSegPoly
// (the partial sum of the ciphertext, nothing stored) and, after the tags are
// checked, kTileSegXor (plaintext of the verified records only).  With
// a.seg_split set, a launch covers the segments [split[c], split[c + 1]) of
// chunk c = a.chunk only (records_kernels.hip: the decrypt pipeline).
// ABL (ablation, tools/ubench only; the product uses 0): 1 = no HBM traffic
// (compute on whatever the LDS holds), 2 = no Poly1305 work.
// NBUF = 2: two LDS tile buffers -- tile t+1's DMA is issued before tile t's
// compute (instead of after it), so it lands during the compute; the wave
// then waits only for it (a counted vmcnt lets tile t-1's stores stay in
// flight).  Twice the LDS: 33 KB per wave at L = 1024, one wave per SIMD.
// kTileSeg*: the per-lane metadata of one segment (from its SegRec); each
// pass loads only what it uses (the Poly1305 pass no key, the XOR pass no r)
struct SegMeta {
  uint32_t k[8], r[4];
  uint32_t nlo, nhi, in_lo, in_hi, out_lo, out_hi, cb, ok, inpl, q;
};
template <int MODE, int SPAN>
__device__ __forceinline__ void seg_meta_load(SegMeta &m, const SegRec *rt, const SegEntry e,
                                              bool valid, const uint8_t *in, const uint8_t *out) {
  constexpr bool XOR = MODE != kTileSegPoly, POLY = MODE != kTileSegXor;
#pragma unroll
  for (int i = 0; i < 8; ++i) m.k[i] = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) m.r[i] = 0u;
  m.nlo = m.nhi = m.in_lo = m.in_hi = m.out_lo = m.out_hi = m.cb = m.ok = m.inpl = m.q = 0u;
  if (valid) {
    const SegRec &R = rt[e.q];
    m.q = e.q;
    const uint64_t io = R.in_off + 1024ull * e.s, oo = R.out_off + 1024ull * e.s;
    m.in_lo = (uint32_t)io; m.in_hi = (uint32_t)(io >> 32);
    m.out_lo = (uint32_t)oo; m.out_hi = (uint32_t)(oo >> 32);
    if (XOR) {
      m.nlo = (uint32_t)R.nonce; m.nhi = (uint32_t)(R.nonce >> 32);
      m.cb = 16u * e.s;
#pragma unroll
      for (int i = 0; i < 8; ++i) m.k[i] = R.k[i];
    }
    if (POLY) {
#pragma unroll
      for (int i = 0; i < 4; ++i) m.r[i] = R.r[i];
    }
    if (MODE == kTileSegXor) {
      m.ok = R.ok;
      m.inpl = in + R.in_off == out + R.out_off;
    }

  }
}

template <bool DECRYPT, int L, bool CONTIG, int MODE = kTileUniform, int ABL = 0, int NBUF = 1,
          int SPAN = 256>
__global__ __launch_bounds__(64) void k_aead_tile(const TileArgs a) {
  using C = TileCfg<L, SPAN>;
  constexpr bool KEYED = MODE != kTileUniform;
  constexpr bool SEG = MODE >= kTileSeg;              // segments of long records
  constexpr bool DO_POLY = MODE != kTileSegXor;       // Poly1305 over the ciphertext
  constexpr bool DO_XOR = MODE != kTileSegPoly;       // keystream XOR + stores
  static_assert(MODE < kTileSegPoly || DECRYPT, "the split segment passes are decrypt's");
  constexpr int OPR = (DECRYPT || SEG) ? C::SPR : C::SPR + 1;  // out pieces / record
  constexpr int OUT_SLOTS = C::RPT * OPR;
  // RECW (contiguous encrypt of records of >= 1 KiB): output instruction
  // q < NDATA stores 64 ciphertext pieces of ONE record (swizzled LDS reads
  // within one 64-slot group: bank-conflict free; destination uniform), the
  // last one the tile's RPT tags.  Otherwise instruction q stores pieces
  // 64q..64q+63 of the tile's output in wire order (ct || tag interleaved).
  // Strided layouts (in-place batches, padded strides) take it too: their
  // wire-order gather (a division by SPR + 1 and a 64-bit address per lane
  // and instruction) pushed the keyed encrypt kernels past 256 VGPRs, i.e.
  // to one wave per SIMD.  Not kTileSeg (RECQ below).
  constexpr bool RECW = !DECRYPT && !SEG && C::SPR >= 64 &&
                        C::SPR % 64 == 0;
  constexpr int NDATA = C::RPT * C::SPR / 64;
  constexpr int NOUT = RECW ? NDATA + 1 : (OUT_SLOTS + 63) / 64;  // store instructions
  static_assert(!(CONTIG && SEG), "segment tiles are strided");
  static_assert(!SEG || (L == 1024 && (SPAN == 256 || SPAN == 128)),
                "segments are 1 KiB, 256 or 128 B per lane");
  static_assert(!SEG || !DO_POLY || SPAN == 256, "the SegRec holds the 256-B spans' powers");
  static_assert(NBUF == 1 || NBUF == 2, "one or two tile buffers");
  // the Poly1305 pass issues the next tile's DMA into buffer 0 itself
  static_assert(MODE != kTileSegPoly || NBUF == 1, "the Poly1305 pass has one tile buffer");
  __shared__ uint4 lds[NBUF * C::NSLOT];
  const uint32_t lane = threadIdx.x;
  const uint8_t *in = a.in;
  uint8_t *out = a.out;
  uint64_t nrec = a.nrec, dbase = 0;
  if (SEG) seg_range(a, dbase, nrec);
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = a.key.w[i];

  const uint32_t rho = lane / C::G, j = lane % C::G;
  // swz(64q + lane) - 64q (glq)
  uint32_t gl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) gl[i] = swz<SPAN>(64u * i + lane) - 64u * i;

  // kTileSeg: each super-tile's per-segment metadata (SegEntry -> SegRec,
  // two dependent loads) is fetched one super-tile ahead -- the SegEntry with
  // the current super-tile's first DMA, the SegRec fields once that DMA has
  // landed -- so its latency hides behind the first tile's compute instead
  // of stalling before every super-tile's first DMA.
  SegMeta nxt;
  SegEntry nxt_e{0u, 0u};
  if (SEG) {
    const uint64_t g = (uint64_t)blockIdx.x * 64 + lane;
    if (g < nrec) nxt_e = a.segs[dbase + g];
    seg_meta_load<MODE, SPAN>(nxt, a.rt, nxt_e, g < nrec, in, out);
  }

  // records per super-tile: 64 (one key lane each)
  constexpr int RPS = 64;
  constexpr int NTS = RPS / C::RPT;  // tiles per super-tile
#pragma unroll 1
  for (uint64_t super0 = (uint64_t)blockIdx.x * RPS; super0 < nrec;
       super0 += (uint64_t)gridDim.x * RPS) {
  // ---- key pass: lane l -> one-time key of record super0 + l -------------
  uint32_t kr[4], kss[4];
  F26 pw[C::LOG2G > 0 && !SEG ? C::LOG2G : 1];  // uniform / keyed: r^BPL, r^(2 BPL), ...
  uint32_t own_q = 0;  // kTileSeg*: the long record of segment super0 + lane
  uint32_t own_k[8], own_nlo = 0, own_nhi = 0;  // keyed modes: this lane's record
  uint32_t own_in_lo = 0, own_in_hi = 0, own_out_lo = 0, own_out_hi = 0;
  uint32_t own_cb = 0;  // kTileSeg: first ChaCha block counter - 1 (16 s)
  bool own_bad = false, own_inplace = false;
  uint32_t own_ok = 1u;  // kTileSegXor: the record's tag verified
  // kTileSegXor: per super-tile, bit l = segment super0 + l's record failed /
  // is decrypted in place (ballots of the lanes' own metadata: no shuffles)
  uint64_t seg_nok = 0, seg_inpl = 0;
  const uint64_t next0 = super0 + (uint64_t)gridDim.x * 64;  // kTileSeg prefetch
  if (SEG) {
#pragma unroll
    for (int i = 0; i < 8; ++i) own_k[i] = nxt.k[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) { kr[i] = nxt.r[i]; kss[i] = 0u; }
    own_q = nxt.q;
    own_nlo = nxt.nlo;
    own_nhi = nxt.nhi;
    own_in_lo = nxt.in_lo; own_in_hi = nxt.in_hi;
    own_out_lo = nxt.out_lo; own_out_hi = nxt.out_hi;
    own_cb = nxt.cb;
    own_ok = nxt.ok;
    own_inplace = nxt.inpl != 0u;
    if (MODE == kTileSegXor) {  // lane l <-> segment super0 + l: wave-uniform masks
      seg_nok = __ballot(own_ok == 0u);
      seg_inpl = __ballot(own_inplace);
    }

    const uint64_t left = nrec - super0;
    tile_load<L, DECRYPT, CONTIG, MODE, ABL, SPAN>(
        NOISE_LDS3(lds), in, a.in_stride, super0,
        left < (uint64_t)C::RPT ? (uint32_t)left : C::RPT, lane, gl, 0u,
        own_in_lo, own_in_hi);
    nxt_e = SegEntry{0u, 0u};
    if (next0 + lane < nrec) nxt_e = a.segs[dbase + next0 + lane];
  } else {
    uint64_t n = a.nonce0 + super0 + lane;
    if (KEYED) {
      const uint64_t rec = super0 + lane;
      uint32_t ki = 0;
      n = 0;
      if (rec < nrec && lane < (uint32_t)RPS) {
        ki = __builtin_nontemporal_load(a.key_idx + rec);  // kTileSessions
        n = __builtin_nontemporal_load(a.nonces + rec);
      }
      own_bad = ki >= a.nkeys;
      if (own_bad) ki = 0;
      const u32x4 *kp = reinterpret_cast<const u32x4 *>(a.keys + 32ull * ki);
      const u32x4 ka = __builtin_nontemporal_load(kp), kb = __builtin_nontemporal_load(kp + 1);
      own_k[0] = ka.x; own_k[1] = ka.y; own_k[2] = ka.z; own_k[3] = ka.w;
      own_k[4] = kb.x; own_k[5] = kb.y; own_k[6] = kb.z; own_k[7] = kb.w;
      // an all-zero row is "no key" (failed handshake split): not processed
      own_bad = own_bad || (ka.x | ka.y | ka.z | ka.w | kb.x | kb.y | kb.z | kb.w) == 0u;
      own_nlo = (uint32_t)n;
      own_nhi = (uint32_t)(n >> 32);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) own_k[i] = k[i];
    }
    // the first tile's DMA goes out before the key pass and lands meanwhile
    {
      const uint64_t left = nrec - super0;
      tile_load<L, DECRYPT, CONTIG, MODE, ABL, SPAN>(
          NOISE_LDS3(lds), in, a.in_stride, super0,
          left < (uint64_t)C::RPT ? (uint32_t)left : C::RPT, lane, gl, 0u,
          own_in_lo, own_in_hi);
    }
    uint32_t otk[16];
    chacha20_block(own_k, 0u, (uint32_t)n, (uint32_t)(n >> 32), otk);
    kr[0] = otk[0] & 0x0fffffffu;
    kr[1] = otk[1] & 0x0ffffffcu;
    kr[2] = otk[2] & 0x0ffffffcu;
    kr[3] = otk[3] & 0x0ffffffcu;
    kss[0] = otk[4]; kss[1] = otk[5]; kss[2] = otk[6]; kss[3] = otk[7];
    if (C::G > 1) {  // r^BPL by squaring (BPL = 8 or 16)
      F26 x = to26(kr[0], kr[1], kr[2], kr[3], 0u);
#pragma unroll
      for (int b = 0; b < C::LOG2BPL; ++b) x = mul26(x, x);
      pw[0] = x;
#pragma unroll
      for (int b = 1; b < C::LOG2G; ++b) pw[b] = mul26(pw[b - 1], pw[b - 1]);
    }
  }
  (void)own_cb;

  bool prev_all = false;  // the previous tile issued all NOUT of its stores
#pragma unroll 1
  for (int t = 0; t < NTS; ++t) {
    const uint64_t rec0 = super0 + (uint64_t)t * C::RPT;
    if (rec0 >= nrec) break;
    const uint32_t nv = (nrec - rec0) < (uint64_t)C::RPT ? (uint32_t)(nrec - rec0) : C::RPT;
    uint4 *lb = lds + ((NBUF == 2 && (t & 1)) ? C::NSLOT : 0);  // this tile's buffer

    // this tile's DMA must have landed.  NBUF = 2: it is older than the
    // previous tile's NOUT stores, which may stay in flight (vmcnt counts
    // loads, stores and LDS-DMA together, in issue order); whenever fewer
    // were issued (partial tile, failed records), wait for everything.
    if (NBUF == 2 && prev_all) wait_vmcnt<NOUT>();
    else wait_vmem();
    wave_lds_fence();
    if (SEG && t == 0) seg_meta_load<MODE, SPAN>(nxt, a.rt, nxt_e, next0 + lane < nrec, in, out);
    // kTileSeg*: this lane's recombination power r^(16 (3 - j)) from its
    // segment's SegRec (lands during the Horner chain below; j = 3: 1)
    F26 own_pw;
    if (SEG && DO_POLY) {
      const uint32_t qs = (uint32_t)__shfl((int)own_q, (int)((uint32_t)t * C::RPT + rho));
      const uint32_t m = C::G - 1u - j, mi = m ? m - 1u : 0u;
      const SegRec &R = a.rt[qs];
      const uint4 v = *reinterpret_cast<const uint4 *>(R.pwlo[mi]);
      const uint32_t v4 = R.pwhi[mi];
      own_pw.a[0] = m ? v.x : 1u; own_pw.a[1] = m ? v.y : 0u; own_pw.a[2] = m ? v.z : 0u;
      own_pw.a[3] = m ? v.w : 0u; own_pw.a[4] = m ? v4 : 0u;
    }
    if (NBUF == 2 && t + 1 < NTS) {  // the next tile's DMA now, into the other buffer
      const uint64_t nrec0 = rec0 + C::RPT;
      if (nrec0 < nrec) {
        const uint64_t left = nrec - nrec0;
        tile_load<L, DECRYPT, CONTIG, MODE, ABL, SPAN>(
            NOISE_LDS3(lds + ((t & 1) ? 0 : C::NSLOT)), in, a.in_stride, nrec0,
            left < (uint64_t)C::RPT ? (uint32_t)left : C::RPT, lane, gl,
            (uint32_t)(t + 1) * C::RPT, own_in_lo, own_in_hi);
      }
    }

    // ---- per-lane record work -------------------------------------------
    const uint32_t src = (uint32_t)t * C::RPT + rho;  // key lane of my record
    Poly1305 p;
    p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
    if (DO_POLY) {
      p.r0 = __shfl(kr[0], src); p.r1 = __shfl(kr[1], src);
      p.r2 = __shfl(kr[2], src); p.r3 = __shfl(kr[3], src);
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      p.s0 = __shfl(kss[0], src); p.s1 = __shfl(kss[1], src);
      p.s2 = __shfl(kss[2], src); p.s3 = __shfl(kss[3], src);
    }

    uint32_t n_lo, n_hi;
    bool bad_key = false;
    uint32_t kt[8];  // this record's key
#pragma unroll
    for (int i = 0; i < 8; ++i) kt[i] = !DO_XOR ? 0u : KEYED ? __shfl(own_k[i], src) : k[i];
    if (KEYED && DO_XOR) {
      n_lo = __shfl(own_nlo, src);
      n_hi = __shfl(own_nhi, src);
      bad_key = __shfl((int)own_bad, src) != 0;
    } else if (!KEYED) {
      const uint64_t n = a.nonce0 + rec0 + rho;
      n_lo = (uint32_t)n;
      n_hi = (uint32_t)(n >> 32);
    } else {  // kTileSegPoly: no keystream
      n_lo = n_hi = 0u;
    }
    // Software pipeline: the ChaCha block of chunk kk+1 is independent of
    // the (serial) Poly1305 chain of chunk kk, so both sit in one basic
    // block and the scheduler interleaves them.
    const uint32_t c0 = j * C::CPL;  // first 64-B chunk of my span (in the record / segment)
    const uint32_t cb = 1u + c0 + (SEG && DO_XOR ? (uint32_t)__shfl((int)own_cb, src) : 0u);  // its counter
    ChaPre pre{};
    uint32_t ks[16];
    if (DO_XOR) {
      pre = chacha_pre(kt, n_lo, n_hi);
      chacha20_block_pre(kt, cb, pre, n_lo, n_hi, ks);
    }
#pragma unroll
    for (int kk = 0; kk < C::CPL; ++kk) {
      const uint32_t c = c0 + kk;
      uint32_t ksn[16];
      if (DO_XOR && kk + 1 < C::CPL) chacha20_block_pre(kt, cb + 1u + kk, pre, n_lo, n_hi, ksn);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t slot = swz<SPAN>(rho * C::SPR + 4u * c + q);
        const uint4 v = lb[slot];
        uint4 o = v;
        if (DO_XOR) {
          o.x = v.x ^ ks[4 * q + 0];
          o.y = v.y ^ ks[4 * q + 1];
          o.z = v.z ^ ks[4 * q + 2];
          o.w = v.w ^ ks[4 * q + 3];
          lb[slot] = o;
        }
        if (!DO_POLY) {
        } else if (ABL == 2) { p.h0 ^= o.x ^ v.y; p.h1 ^= o.z ^ v.w; }
        else if (DECRYPT) poly_block(p, v.x, v.y, v.z, v.w);
        else poly_block(p, o.x, o.y, o.z, o.w);
      }
      if (DO_XOR && kk + 1 < C::CPL) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] = ksn[i];
      }
    }
    if (C::G > 1 && DO_POLY) {
      // acc_j * r^(BPL (G-1-j)), then sum over the record's G lanes
      F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
      if (SEG) {
        h = mul26(h, own_pw);
      } else {
        const uint32_t m = C::G - 1 - j;
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
      }
#pragma unroll
      for (int b = 0; b < C::LOG2G; ++b) {
        // limbs are < 2^26 + 2^9 after mul26: 16 of them fit in 32 bits,
        // 64 do not, so wide records re-normalise halfway
        if (b == 4) carry26(h);
#pragma unroll
        for (int i = 0; i < 5; ++i) h.a[i] += __shfl_xor(h.a[i], 1 << b);
      }
      carry26(h);
      carry26(h);
      from26(h, p.h0, p.h1, p.h2, p.h3, p.h4);
    }
    uint32_t tag[4] = {0u, 0u, 0u, 0u};
    const bool valid = rho < nv;
    if (SEG) {
      // the segment's partial sum (no length block, no s); lane 0 of the
      // segment stores it
      if (DO_POLY && j == 0 && valid) {
        const u32x4 w0 = {p.h0, p.h1, p.h2, p.h3};
        const uint64_t g = dbase + super0 + (uint64_t)t * C::RPT + rho;
        __builtin_nontemporal_store(w0, (g_u32x4 *)(a.partial + g));
        __builtin_nontemporal_store(p.h4, (__attribute__((address_space(1))) uint32_t *)(a.partial_hi + g));
      }
    } else {
      poly_block(p, 0u, 0u, (uint32_t)L, 0u);  // LE64(ad_len = 0) || LE64(L)
      poly_final(p, tag);
    }
    uint64_t fail_mask = 0;  // bit (r * G): record r of this tile is not output
    const uint64_t badk_mask = KEYED ? __ballot(j == 0 && bad_key) : 0ull;
    fail_mask = badk_mask;
    // cross-lane reads stay outside divergent code: a ds_bpermute from a lane
    // that is inactive does not return that lane's value
    constexpr bool PER_REC_INPL = MODE == kTileSegXor;
    uint64_t inpl_seg = 0;  // kTileSegXor: bit r * G = slot r is in place
    if (MODE == kTileSegXor) {
      // a segment of a record whose tag failed: not output as computed.  Slot
      // r of tile t is segment super0 + t RPT + r: bit t RPT + r of the masks
      const uint32_t nok = (uint32_t)(seg_nok >> (t * C::RPT)), ip = (uint32_t)(seg_inpl >> (t * C::RPT));
#pragma unroll
      for (int r = 0; r < C::RPT; ++r) {
        fail_mask |= (uint64_t)((nok >> r) & 1u) << (r * C::G);
        inpl_seg |= (uint64_t)((ip >> r) & 1u) << (r * C::G);
      }
    } else if (SEG) {
    } else if (DECRYPT) {
      const uint4 want = lb[C::REC_SLOTS + rho];
      const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) |
                            (want.z ^ tag[2]) | (want.w ^ tag[3]);
      fail_mask |= __ballot(j == 0 && diff != 0u);
      if (j == 0 && valid) {
        a.status[rec0 + rho] = bad_key ? 2u : (diff ? 1u : 0u);
      }
    } else if (j == 0) {
      lb[C::REC_SLOTS + rho] = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    }
    // kTileSegXor: a failed in-place record is kept, a failed copy is zeroed
    const uint64_t inpl_mask = MODE == kTileSegXor ? inpl_seg : 0ull;
    wave_lds_fence();
    if (!DO_XOR) {  // kTileSegPoly: nothing to store; the next tile's DMA
      prev_all = false;
      if (t + 1 < NTS) {
        const uint64_t nrec0 = rec0 + C::RPT;
        if (nrec0 < nrec) {
          wait_lds();  // this tile's LDS reads done before the DMA overwrites them
          wave_lds_fence();
          const uint64_t left = nrec - nrec0;
          tile_load<L, DECRYPT, CONTIG, MODE, ABL, SPAN>(
              NOISE_LDS3(lds), in, a.in_stride, nrec0,
              left < (uint64_t)C::RPT ? (uint32_t)left : C::RPT, lane, gl,
              (uint32_t)(t + 1) * C::RPT, own_in_lo, own_in_hi);
        }
      }
      continue;
    }

    // ---- gather this tile's output records into registers, store them --
    // Keyed modes gather and store in NPART parts: 17 uint4 pieces live at
    // once (L >= 512 encrypt) push those kernels past 256 VGPRs into AGPR
    // and SGPR spills.  The next tile's DMA overwrites the LDS, so it goes
    // out after the last part's gather (before that part's stores).
    constexpr int NPART = (KEYED && NBUF == 1 && NOUT > 8) ? 2 : 1;
    constexpr int NQ = (NOUT + NPART - 1) / NPART;
    const bool full = nv == (uint32_t)C::RPT;
    // RECQ (segments): output instruction q < NDATA holds the 64 data pieces
    // of KiB q % (SPR / 64) of record q / (SPR / 64) (uniform destination,
    // v_readlane), instruction NDATA (encrypt) the RPT tags
    constexpr bool RECQ = SEG;
    auto piece = [&](int q, uint32_t &r, uint32_t &pc, uint32_t &slot, bool &ok) {
      if constexpr (RECW) {
        if (q < NDATA) {
          r = (uint32_t)q / (C::SPR / 64);
          pc = 64u * ((uint32_t)q % (C::SPR / 64)) + lane;
          slot = swz<SPAN>(64u * q + lane);  // == swz(r * SPR + pc)
          ok = true;
        } else {
          r = lane < (uint32_t)C::RPT ? lane : 0u;
          pc = C::SPR;
          slot = C::REC_SLOTS + r;
          ok = lane < (uint32_t)C::RPT;
        }
        return;
      }
      if (RECQ) {
        if (q < NDATA) {
          r = (uint32_t)q / (C::SPR / 64);
          pc = 64u * ((uint32_t)q % (C::SPR / 64)) + lane;
          slot = swz<SPAN>(64u * q + lane);
          ok = true;
        } else {
          r = lane < (uint32_t)C::RPT ? lane : 0u; pc = C::SPR; slot = C::REC_SLOTS + r;
          ok = lane < (uint32_t)C::RPT;
        }
        return;
      }
      const uint32_t g = 64u * q + lane;  // output piece (record r, piece pc)
      r = g / OPR;
      pc = g % OPR;
      if (CONTIG && DECRYPT) slot = 64u * q + glq<SPAN>(gl, q);  // == swz(g)
      else slot = pc < (uint32_t)C::SPR ? swz<SPAN>(r * C::SPR + pc) : C::REC_SLOTS + r;
      ok = OUT_SLOTS % 64 == 0 || g < (uint32_t)OUT_SLOTS;
    };
#pragma unroll
    for (int part = 0; part < NPART; ++part) {
      const int q0 = part * NQ;
      uint4 ov[NQ];
      bool st[NQ];
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int q = q0 + qq;
        if (q >= NOUT) break;
        uint32_t r, pc, slot;
        bool ok;
        piece(q, r, pc, slot, ok);
        st[qq] = ok && (full || r < nv);
        ov[qq] = lb[slot < (uint32_t)C::NSLOT ? slot : 0u];
      }
      // Records that must not be output as computed (rare; a separate,
      // wave-uniform branch so the common path carries none of this):
      // failed tag (decrypt): keep an in-place record, zero a copy; invalid
      // key index: write nothing.
      if ((DECRYPT || KEYED) && fail_mask != 0) {
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const int q = q0 + qq;
          if (q >= NOUT) break;
          uint32_t r, pc, slot;
          bool ok;
          piece(q, r, pc, slot, ok);
          if ((fail_mask >> (r * C::G)) & 1u) {
            const bool bad_key_rec = KEYED && ((badk_mask >> (r * C::G)) & 1u);
            const bool inpl = PER_REC_INPL ? ((inpl_mask >> (r * C::G)) & 1u) != 0
                                           : a.in_place != 0;
            st[qq] = st[qq] && DECRYPT && !inpl && !bad_key_rec;
            ov[qq] = make_uint4(0u, 0u, 0u, 0u);
          }
        }
      }
      if (part == NPART - 1) {
        wait_lds();  // LDS reads done
        wave_lds_fence();
        // ---- NBUF = 1: next tile's DMA, then these stores, both in flight
        if (NBUF == 1 && t + 1 < NTS) {
          const uint64_t nrec0 = rec0 + C::RPT;
          if (nrec0 < nrec) {
            const uint64_t left = nrec - nrec0;
            tile_load<L, DECRYPT, CONTIG, MODE, ABL, SPAN>(
                NOISE_LDS3(lds), in, a.in_stride, nrec0,
                left < (uint64_t)C::RPT ? (uint32_t)left : C::RPT, lane, gl,
                (uint32_t)(t + 1) * C::RPT, own_in_lo, own_in_hi);
          }
        }
      }
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int q = q0 + qq;
        if (q >= NOUT) break;
        const uint32_t g = 64u * q + lane;
        uint32_t r, pc, slot;
        bool ok;
        piece(q, r, pc, slot, ok);
        bool store = st[qq];
        if (ABL == 1) store = store && (ov[qq].x == 0x12345678u && ov[qq].y == 0x9abcdef0u);
        uint8_t *dst;
        if (RECQ && q < NDATA) {  // output instruction q: a KiB of one record / segment: uniform offset
          const uint32_t kl = (uint32_t)t * C::RPT + (uint32_t)q / (C::SPR / 64);
          const uint64_t off = join64((uint32_t)__builtin_amdgcn_readlane((int)own_out_hi, (int)kl),
                                      (uint32_t)__builtin_amdgcn_readlane((int)own_out_lo, (int)kl));
          dst = out + off + 16u * pc;
        } else {
          dst = out + rec0 * a.out_stride +
                ((CONTIG && !RECW) ? 16ull * g : r * a.out_stride + 16u * pc);
        }
        if (store) store16<true>(dst, ov[qq], 16);
      }
    }
    prev_all = ABL == 0 && full && fail_mask == 0;
  }
  }  // super-tiles
}

}  // namespace noise_amd
