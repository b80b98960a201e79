// chachapoly_device.hpp -- gfx950 device arithmetic for the Noise ChaChaPoly
// record engine: ChaCha20 block function, Poly1305 block/finalise, and the
// per-record AEAD walk (Noise nonce framing, ct || tag layout).
//
// Mapping (DESIGN.md "Kernels"): ONE LANE = ONE RECORD.  A lane derives its
// record's one-time Poly1305 key from ChaCha block 0, then walks the record
// in 64-byte chunks: ChaCha block (1 + chunk) -> XOR -> 4 Poly1305 blocks.
// Everything stays in VGPRs; nothing is shared between lanes, so there is
// no LDS, no barrier and no cross-lane reduction.  This is the op-minimal
// mapping: 1 KiB costs exactly 17 ChaCha blocks + 65 Poly1305 blocks per
// record, with no r-power precomputation (a k-lane split of one record's
// Poly1305 would need r^2..r^k per record, +30-120 % Poly work).
//
// Arithmetic references:
//   ChaCha20 quarter-round / 20 rounds   monocypher.c:169-200 (what is computed)
//   keystream feed-forward, counter      monocypher.c:219-253 (what is computed)
//   Poly1305 clamp                        monocypher.c:366-375
//   Poly1305 block (poly_block)           monocypher.c:314-357 -- also the
//     formulation: the radix-2^32 limbs, rr_j = r_j + (r_j >> 2), the
//     five-term column sums and the fold of the bits above 2^130 (the carry
//     handling here is this build's own: full carries at the add)
//   Poly1305 final (poly_final)           monocypher.c:426-438 (formulation too)
//   AEAD layout ad|pad|ct|pad|lens       monocypher.c:2858-2873
//   Noise nonce 0^32 || LE64(n)          noise.cpp:207-215
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace noise_amd {

// A 32-byte key passed by value as a kernel argument (lands in SGPRs).
struct KeyArg {
  uint32_t w[8];
};

// "expand 32-byte k"
constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu,
                   kSigma2 = 0x79622d32u, kSigma3 = 0x6b206574u;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) {
  // one v_alignbit_b32
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

#define NOISE_QR(a, b, c, d)              \
  a += b; d = rotl32(d ^ a, 16);          \
  c += d; b = rotl32(b ^ c, 12);          \
  a += b; d = rotl32(d ^ a, 8);           \
  c += d; b = rotl32(b ^ c, 7);

// Lane i of a 4-lane quad <- lane (i + n) mod 4 of the quad (DPP quad_perm:
// one v_mov_b32_dpp, no LDS).
template <int N>
__device__ __forceinline__ uint32_t quad_rot(uint32_t x) {
  constexpr int perm = ((0 + N) & 3) | (((1 + N) & 3) << 2) | (((2 + N) & 3) << 4) |
                       (((3 + N) & 3) << 6);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, perm, 0xf, 0xf, false);
}

// ChaCha20 block on a QUAD of lanes (the latency kernel): lane q of the quad
// holds column q of the 4x4 state -- rows a (constant q), b (key word q),
// c (key word 4 + q), d (word 12 + q: counter, 0, n_lo, n_hi).  A column
// round is one quarter round per lane; the diagonal round first rotates b,
// c, d by 1, 2, 3 lanes (DPP), so lane q works on diagonal q, then rotates
// them back.  The dependent chain is 20 quarter rounds + 60 DPP moves instead
// of one lane's 80 quarter rounds: ~3x lower latency for one block, the
// same instruction count per block (monocypher.c:178-200, RFC 8439 2.3).
// out[r] = keystream word 4r + q (after the feed-forward add).
__device__ __forceinline__ void chacha20_quad(const uint32_t k[8], uint32_t q, uint32_t ctr,
                                              uint32_t n_lo, uint32_t n_hi, uint32_t out[4]) {
  uint32_t a = q == 0 ? kSigma0 : q == 1 ? kSigma1 : q == 2 ? kSigma2 : kSigma3;
  uint32_t b = q == 0 ? k[0] : q == 1 ? k[1] : q == 2 ? k[2] : k[3];
  uint32_t c = q == 0 ? k[4] : q == 1 ? k[5] : q == 2 ? k[6] : k[7];
  uint32_t d = q == 0 ? ctr : q == 1 ? 0u : q == 2 ? n_lo : n_hi;
  const uint32_t a0 = a, b0 = b, c0 = c, d0 = d;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    NOISE_QR(a, b, c, d)
    b = quad_rot<1>(b);
    c = quad_rot<2>(c);
    d = quad_rot<3>(d);
    NOISE_QR(a, b, c, d)
    b = quad_rot<3>(b);
    c = quad_rot<2>(c);
    d = quad_rot<1>(d);
  }
  out[0] = a + a0;
  out[1] = b + b0;
  out[2] = c + c0;
  out[3] = d + d0;
}

// ChaCha20 block with IETF word layout: x12 = block counter, x13 = 0 (the
// four zero bytes of the Noise nonce), x14/x15 = lo/hi 32 bits of n.
// ks[] receives the 16 keystream words (after the feed-forward add).
// When k[] and ctr are wave-uniform (single-key batches) the compiler keeps
// them in SGPRs and the first-round columns 0/1 run on the scalar unit.
__device__ __forceinline__ void chacha20_block(const uint32_t k[8],
                                               uint32_t ctr, uint32_t n_lo,
                                               uint32_t n_hi, uint32_t ks[16]) {
  uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
  uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = ctr, x13 = 0, x14 = n_lo, x15 = n_hi;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    NOISE_QR(x0, x4, x8, x12)
    NOISE_QR(x1, x5, x9, x13)
    NOISE_QR(x2, x6, x10, x14)
    NOISE_QR(x3, x7, x11, x15)
    NOISE_QR(x0, x5, x10, x15)
    NOISE_QR(x1, x6, x11, x12)
    NOISE_QR(x2, x7, x8, x13)
    NOISE_QR(x3, x4, x9, x14)
  }
  ks[0] = x0 + kSigma0;  ks[1] = x1 + kSigma1;
  ks[2] = x2 + kSigma2;  ks[3] = x3 + kSigma3;
  ks[4] = x4 + k[0];     ks[5] = x5 + k[1];
  ks[6] = x6 + k[2];     ks[7] = x7 + k[3];
  ks[8] = x8 + k[4];     ks[9] = x9 + k[5];
  ks[10] = x10 + k[6];   ks[11] = x11 + k[7];
  ks[12] = x12 + ctr;    ks[13] = x13;
  ks[14] = x14 + n_lo;   ks[15] = x15 + n_hi;
}

// Round-1 columns 1, 2 and 3 depend only on (key, nonce), not on the block
// counter, so a lane that runs several blocks of one record computes them
// once (chacha_pre) and starts each block from them (chacha20_block_pre):
// 3 of the 80 quarter-rounds per block saved (column 1 -- x13 = 0 -- is
// wave-uniform for a single key and then runs on the scalar unit anyway).
struct ChaPre {
  uint32_t x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15;
};

__device__ __forceinline__ ChaPre chacha_pre(const uint32_t k[8], uint32_t n_lo,
                                             uint32_t n_hi) {
  ChaPre p;
  p.x1 = kSigma1; p.x5 = k[1]; p.x9 = k[5]; p.x13 = 0u;
  p.x2 = kSigma2; p.x6 = k[2]; p.x10 = k[6]; p.x14 = n_lo;
  p.x3 = kSigma3; p.x7 = k[3]; p.x11 = k[7]; p.x15 = n_hi;
  NOISE_QR(p.x1, p.x5, p.x9, p.x13)
  NOISE_QR(p.x2, p.x6, p.x10, p.x14)
  NOISE_QR(p.x3, p.x7, p.x11, p.x15)
  return p;
}

__device__ __forceinline__ void chacha20_block_pre(const uint32_t k[8],
                                                   uint32_t ctr,
                                                   const ChaPre &pre,
                                                   uint32_t n_lo, uint32_t n_hi,
                                                   uint32_t ks[16]) {
  uint32_t x0 = kSigma0, x1 = pre.x1, x2 = pre.x2, x3 = pre.x3;
  uint32_t x4 = k[0], x5 = pre.x5, x6 = pre.x6, x7 = pre.x7;
  uint32_t x8 = k[4], x9 = pre.x9, x10 = pre.x10, x11 = pre.x11;
  uint32_t x12 = ctr, x13 = pre.x13, x14 = pre.x14, x15 = pre.x15;
  // round 1: column 0 (the only counter-dependent one), then diagonals
  NOISE_QR(x0, x4, x8, x12)
  NOISE_QR(x0, x5, x10, x15)
  NOISE_QR(x1, x6, x11, x12)
  NOISE_QR(x2, x7, x8, x13)
  NOISE_QR(x3, x4, x9, x14)
#pragma unroll
  for (int i = 1; i < 10; ++i) {
    NOISE_QR(x0, x4, x8, x12)
    NOISE_QR(x1, x5, x9, x13)
    NOISE_QR(x2, x6, x10, x14)
    NOISE_QR(x3, x7, x11, x15)
    NOISE_QR(x0, x5, x10, x15)
    NOISE_QR(x1, x6, x11, x12)
    NOISE_QR(x2, x7, x8, x13)
    NOISE_QR(x3, x4, x9, x14)
  }
  ks[0] = x0 + kSigma0;  ks[1] = x1 + kSigma1;
  ks[2] = x2 + kSigma2;  ks[3] = x3 + kSigma3;
  ks[4] = x4 + k[0];     ks[5] = x5 + k[1];
  ks[6] = x6 + k[2];     ks[7] = x7 + k[3];
  ks[8] = x8 + k[4];     ks[9] = x9 + k[5];
  ks[10] = x10 + k[6];   ks[11] = x11 + k[7];
  ks[12] = x12 + ctr;    ks[13] = x13;
  ks[14] = x14 + n_lo;   ks[15] = x15 + n_hi;
}

// Poly1305 in radix 2^32 (four 32-bit limbs + a small 2^128 limb), which
// turns each block into 20 v_mad_u64_u32 + ~15 add/carry ops.  The clamp
// makes r1..r3 multiples of 4, so 2^128 * r_j == 5 * (r_j / 4) (mod p)
// folds the high partial products back with rr_j = r_j + (r_j >> 2).
struct Poly1305 {
  uint32_t h0, h1, h2, h3, h4;
  uint32_t r0, r1, r2, r3;
  uint32_t rr0, rr1, rr2, rr3;  // rr0 = 5*(r0>>2); rr_j = 5*(r_j/4)
  uint32_t r0lo;                // r0 & 3
  uint32_t s0, s1, s2, s3;      // the "s" half of the one-time key
};

// one-time key = keystream block 0 words 0..7 (monocypher.c:2903, 366-375)
__device__ __forceinline__ void poly_init(Poly1305 &p, const uint32_t otk[16]) {
  p.r0 = otk[0] & 0x0fffffffu;
  p.r1 = otk[1] & 0x0ffffffcu;
  p.r2 = otk[2] & 0x0ffffffcu;
  p.r3 = otk[3] & 0x0ffffffcu;
  p.rr0 = (p.r0 >> 2) * 5u;
  p.rr1 = p.r1 + (p.r1 >> 2);
  p.rr2 = p.r2 + (p.r2 >> 2);
  p.rr3 = p.r3 + (p.r3 >> 2);
  p.r0lo = p.r0 & 3u;
  p.s0 = otk[4]; p.s1 = otk[5]; p.s2 = otk[6]; p.s3 = otk[7];
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}

// h <- (h + m + 2^128) * r  (partially reduced: h4 <= 4 on exit).
// Written with explicit 32-bit carry chains (v_add_co / v_addc_co) so the
// compiler never widens limbs to 64 bits: 5 + 20 mad64 + ~10 ops per block.
__device__ __forceinline__ void poly_block(Poly1305 &p, uint32_t m0,
                                           uint32_t m1, uint32_t m2,
                                           uint32_t m3) {
  unsigned c;
  // s = h + m + 2^128 with full carry propagation (s4 <= 6)
  const uint32_t s0 = __builtin_addc(p.h0, m0, 0u, &c);
  const uint32_t s1 = __builtin_addc(p.h1, m1, c, &c);
  const uint32_t s2 = __builtin_addc(p.h2, m2, c, &c);
  const uint32_t s3 = __builtin_addc(p.h3, m3, c, &c);
  const uint32_t s4 = p.h4 + c + 1u;
  // column sums, each < 2^63
  const uint64_t x0 = mad64(s0, p.r0, mad64(s1, p.rr3, mad64(s2, p.rr2, mad64(s3, p.rr1, mad64(s4, p.rr0, 0)))));
  const uint64_t x1 = mad64(s0, p.r1, mad64(s1, p.r0, mad64(s2, p.rr3, mad64(s3, p.rr2, mad64(s4, p.rr1, 0)))));
  const uint64_t x2 = mad64(s0, p.r2, mad64(s1, p.r1, mad64(s2, p.r0, mad64(s3, p.rr3, mad64(s4, p.rr2, 0)))));
  const uint64_t x3 = mad64(s0, p.r3, mad64(s1, p.r2, mad64(s2, p.r1, mad64(s3, p.r0, mad64(s4, p.rr3, 0)))));
  const uint32_t x4 = __umul24(s4, p.r0lo);  // tiny * tiny
  // partial reduction: fold everything at and above 2^130 back as *5
  const uint32_t u5 = x4 + (uint32_t)(x3 >> 32);
  const uint32_t q = u5 >> 2;
  p.h0 = __builtin_addc(q + (q << 2), (uint32_t)x0, 0u, &c);
  p.h1 = __builtin_addc((uint32_t)x1, (uint32_t)(x0 >> 32), c, &c);
  p.h2 = __builtin_addc((uint32_t)x2, (uint32_t)(x1 >> 32), c, &c);
  p.h3 = __builtin_addc((uint32_t)x3, (uint32_t)(x2 >> 32), c, &c);
  p.h4 = (u5 & 3u) + c;
}

// tag = (h mod 2^130-5) + s  mod 2^128  (monocypher.c:424-436)
__device__ __forceinline__ void poly_final(const Poly1305 &p, uint32_t tag[4]) {
  // carry of h + 5 into bit 130 says whether h >= p
  uint64_t c = 5;
  c = (c + p.h0) >> 32;
  c = (c + p.h1) >> 32;
  c = (c + p.h2) >> 32;
  c = (c + p.h3) >> 32;
  c += p.h4;
  c = (c >> 2) * 5;  // 0 or 5
  c += (uint64_t)p.h0 + p.s0;
  tag[0] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)p.h1 + p.s1;
  tag[1] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)p.h2 + p.s2;
  tag[2] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)p.h3 + p.s3;
  tag[3] = (uint32_t)c;
}

// ------------------------------------------------ general Poly1305 products
// Radix-2^26 arithmetic for multiplying by an arbitrary element (powers of
// r are not "clamped", so the radix-2^32 shortcut above does not apply).
// Used only to recombine a record's per-lane partial Horner sums
// (O(log G) products per lane per record), never in the per-block loop.
constexpr uint32_t kM26 = 0x3ffffffu;

struct F26 {
  uint32_t a[5];
};

__device__ __forceinline__ F26 to26(uint32_t h0, uint32_t h1, uint32_t h2,
                                    uint32_t h3, uint32_t h4) {
  F26 f;
  f.a[0] = h0 & kM26;
  f.a[1] = __builtin_amdgcn_alignbit(h1, h0, 26) & kM26;
  f.a[2] = __builtin_amdgcn_alignbit(h2, h1, 20) & kM26;
  f.a[3] = __builtin_amdgcn_alignbit(h3, h2, 14) & kM26;
  f.a[4] = (h3 >> 8) | (h4 << 24);
  return f;
}

// value (any limb sizes < 2^31) -> radix 2^32 words h0..h3 and small h4
__device__ __forceinline__ void from26(const F26 &f, uint32_t &h0, uint32_t &h1,
                                       uint32_t &h2, uint32_t &h3, uint32_t &h4) {
  uint64_t w = (uint64_t)f.a[0] + ((uint64_t)f.a[1] << 26);
  h0 = (uint32_t)w;
  w = (w >> 32) + ((uint64_t)f.a[2] << 20);
  h1 = (uint32_t)w;
  w = (w >> 32) + ((uint64_t)f.a[3] << 14);
  h2 = (uint32_t)w;
  w = (w >> 32) + ((uint64_t)f.a[4] << 8);
  h3 = (uint32_t)w;
  h4 = (uint32_t)(w >> 32);
}

// full carry propagation modulo 2^130-5 (limbs < 2^31 in, < 2^26(+1) out)
__device__ __forceinline__ void carry26(F26 &f) {
  uint32_t c;
  c = f.a[0] >> 26; f.a[0] &= kM26; f.a[1] += c;
  c = f.a[1] >> 26; f.a[1] &= kM26; f.a[2] += c;
  c = f.a[2] >> 26; f.a[2] &= kM26; f.a[3] += c;
  c = f.a[3] >> 26; f.a[3] &= kM26; f.a[4] += c;
  c = f.a[4] >> 26; f.a[4] &= kM26; f.a[0] += c * 5u;
  c = f.a[0] >> 26; f.a[0] &= kM26; f.a[1] += c;
}

// x * y mod 2^130-5; x limbs < 2^27, y limbs < 2^26 (+1)
__device__ __forceinline__ F26 mul26(const F26 &x, const F26 &y) {
  const uint32_t y1 = y.a[1] * 5u, y2 = y.a[2] * 5u, y3 = y.a[3] * 5u,
                 y4 = y.a[4] * 5u;
  const uint32_t *a = x.a, *b = y.a;
  uint64_t d0 = mad64(a[0], b[0], mad64(a[1], y4, mad64(a[2], y3, mad64(a[3], y2, mad64(a[4], y1, 0)))));
  uint64_t d1 = mad64(a[0], b[1], mad64(a[1], b[0], mad64(a[2], y4, mad64(a[3], y3, mad64(a[4], y2, 0)))));
  uint64_t d2 = mad64(a[0], b[2], mad64(a[1], b[1], mad64(a[2], b[0], mad64(a[3], y4, mad64(a[4], y3, 0)))));
  uint64_t d3 = mad64(a[0], b[3], mad64(a[1], b[2], mad64(a[2], b[1], mad64(a[3], b[0], mad64(a[4], y4, 0)))));
  uint64_t d4 = mad64(a[0], b[4], mad64(a[1], b[3], mad64(a[2], b[2], mad64(a[3], b[1], mad64(a[4], b[0], 0)))));
  F26 r;
  uint32_t c;
  c = (uint32_t)(d0 >> 26); r.a[0] = (uint32_t)d0 & kM26; d1 += c;
  c = (uint32_t)(d1 >> 26); r.a[1] = (uint32_t)d1 & kM26; d2 += c;
  c = (uint32_t)(d2 >> 26); r.a[2] = (uint32_t)d2 & kM26; d3 += c;
  c = (uint32_t)(d3 >> 26); r.a[3] = (uint32_t)d3 & kM26; d4 += c;
  c = (uint32_t)(d4 >> 26); r.a[4] = (uint32_t)d4 & kM26;
  const uint64_t t = (uint64_t)c * 5u + r.a[0];  // c < 2^32, so widen
  r.a[0] = (uint32_t)t & kM26;
  r.a[1] += (uint32_t)(t >> 26);
  return r;
}

// ---------------------------------------------------------------- memory
// Wave-uniform 32-bit value into an SGPR.  The builtin returns a signed
// int: widening it directly sign-extends (an offset >= 2^31 would turn
// into a wild address), so it is always taken as uint32_t here.
__device__ __forceinline__ uint32_t uniform32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint64_t join64(uint32_t hi, uint32_t lo) {
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}

// Explicit memory waits (s_waitcnt simm16, gfx9 layout: vmcnt in [3:0] and
// [15:14], expcnt [6:4], lgkmcnt [11:8]; a field at its maximum = no wait).
// Callers follow each with wave_lds_fence() to pin LDS accesses around it.
__device__ __forceinline__ void wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)
__device__ __forceinline__ void wait_lds() { __builtin_amdgcn_s_waitcnt(0xC07F); }   // lgkmcnt(0)
__device__ __forceinline__ void wait_all() { __builtin_amdgcn_s_waitcnt(0x0070); }   // both
// vmcnt(N): all but the wave's N youngest vector-memory operations done
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);  // expcnt, lgkmcnt: no wait
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Record buffers are device (global) memory.  Naming the address space keeps
// the compiler from falling back to FLAT instructions when it cannot trace a
// pointer to a kernel argument (e.g. base + an offset read from a
// descriptor); FLAT stores also count against lgkmcnt.
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

// LDS-DMA of 16 bytes per lane: global -> LDS at lds_base + 16 * lane
// (global_load_lds_dwordx4, M0 = the wave-uniform LDS byte address).  Issued
// from inline asm so that the compiler does not see an LDS write in flight:
// otherwise it drains vmcnt(0) before the first ds_read of ANY part of the
// LDS array, which would serialise a DMA into the other tile buffer with the
// compute on this one.  Every reader of a DMA'd buffer therefore waits with
// an explicit s_waitcnt vmcnt (wait_vmem / wait_vmcnt) and a wave fence.
// sbase: wave-uniform 64-bit base (SGPRs) + per-lane 32-bit offset; vaddr:
// per-lane 64-bit address.  Host builds (tools/emu) use the builtin.
typedef __attribute__((address_space(3))) void lds_void;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// The record DMAs stream (the nt policy: each byte is read once).  Same box,
// six alternating runs each (round 4, profiles/round4/ab/dma_nt.md): config 2
// +0.0..+2.3 %, config 4 +0.9..+2.6 %, every run faster; "sc1 nt" and
// "sc0 sc1 nt" were no better, and the default policy on the decrypt's
// Poly1305 pass (whose ciphertext the keystream pass reads again) was no
// faster at 4..64 chunks (round 5, profiles/round5/ab/cfg4_chunks_policy.txt).
__device__ __forceinline__ void lds_dma16_s(const void *sbase, uint32_t voff, lds_void *lds_base) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NOISE_DMA_BUILTIN)
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt"
               :: "v"(voff), "s"(sbase), "s"((uint32_t)(uintptr_t)lds_base) : "memory", "m0");
#else
  __builtin_amdgcn_global_load_lds((const void *)((const uint8_t *)sbase + voff), lds_base, 16, 0, 0);
#endif
}
__device__ __forceinline__ void lds_dma16_v(const void *vaddr, lds_void *lds_base) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NOISE_DMA_BUILTIN)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt"
               :: "v"(vaddr), "s"((uint32_t)(uintptr_t)lds_base) : "memory", "m0");
#else
  __builtin_amdgcn_global_load_lds(vaddr, lds_base, 16, 0, 0);
#endif
}
// The same with system-scope cache bypass (sc0 sc1): for host-mapped memory
// that the host rewrites while a resident kernel keeps running (no kernel
// start invalidates the GPU caches between requests there; a plain load can
// hit a stale line of the previous request).
__device__ __forceinline__ void lds_dma16_v_sys(const void *vaddr, lds_void *lds_base) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NOISE_DMA_BUILTIN)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc0 sc1"
               :: "v"(vaddr), "s"((uint32_t)(uintptr_t)lds_base) : "memory", "m0");
#else
  __builtin_amdgcn_global_load_lds(vaddr, lds_base, 16, 0, 1 | 16);
#endif
}
#pragma clang diagnostic pop

// Byte-granular little-endian word load/store for unaligned records.
__device__ __forceinline__ uint32_t ld_bytes(const uint8_t *p, int n) {
  uint32_t w = 0;
  for (int i = 0; i < n; ++i) w |= (uint32_t)p[i] << (8 * i);
  return w;
}
__device__ __forceinline__ void st_bytes(uint8_t *p, uint32_t w, int n) {
  for (int i = 0; i < n; ++i) p[i] = (uint8_t)(w >> (8 * i));
}

// Load `n` (0..16) bytes as 4 LE words, zero padded.  VEC: the 16 bytes
// are 16-byte aligned and readable (n == 16 whenever VEC is used).
template <bool VEC>
__device__ __forceinline__ uint4 load16(const uint8_t *p, int n) {
  if (VEC) {
    // one global_load_dwordx4; records are streamed once (nontemporal)
    const u32x4 w = __builtin_nontemporal_load((const g_u32x4 *)p);
    return make_uint4(w.x, w.y, w.z, w.w);
  }
  uint4 v;
  v.x = ld_bytes(p, n >= 4 ? 4 : n);
  v.y = n > 4 ? ld_bytes(p + 4, n >= 8 ? 4 : n - 4) : 0u;
  v.z = n > 8 ? ld_bytes(p + 8, n >= 12 ? 4 : n - 8) : 0u;
  v.w = n > 12 ? ld_bytes(p + 12, n - 12) : 0u;
  return v;
}
template <bool VEC>
__device__ __forceinline__ void store16(uint8_t *p, uint4 v, int n) {
#if defined(NOISE_HIP_EMU)
  if (emu::store_hook) emu::store_hook(p, &v, VEC ? 16 : n);  // tools/emu: every record store seen
#endif
  if (VEC) {
    // one aligned global_store_dwordx4 (a plain uint4 store may be
    // re-split by the store merger into misaligned dwordx3/x4 pieces)
    const u32x4 w = {v.x, v.y, v.z, v.w};
    // nt: round 4 same-box A/B against plain stores, config 2 +0.4..+1.6 %,
    // config 4 +1.8..+4.2 % (profiles/round4/ab/dma_nt.md)
    __builtin_nontemporal_store(w, (g_u32x4 *)p);
    return;
  }
  st_bytes(p, v.x, n >= 4 ? 4 : n);
  if (n > 4) st_bytes(p + 4, v.y, n >= 8 ? 4 : n - 4);
  if (n > 8) st_bytes(p + 8, v.z, n >= 12 ? 4 : n - 8);
  if (n > 12) st_bytes(p + 12, v.w, n - 12);
}

// Keep the first `n` (0..16) bytes of a 16-byte piece, zero the rest (the
// keystream past a record's end must not reach the MAC).
__device__ __forceinline__ uint4 mask_bytes(uint4 v, int n) {
  uint32_t m[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int b = n - 4 * w;
    m[w] = b >= 4 ? 0xffffffffu : b <= 0 ? 0u : (1u << (8 * b)) - 1u;
  }
  return make_uint4(v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]);
}

// Poly1305 over `n` bytes of associated data, zero padded to 16.
__device__ __forceinline__ void poly_ad(Poly1305 &p, const uint8_t *ad,
                                        uint32_t n) {
  for (uint32_t off = 0; off < n; off += 16) {
    const int m = (n - off) >= 16 ? 16 : (int)(n - off);
    const uint4 v = load16<false>(ad + off, m);
    poly_block(p, v.x, v.y, v.z, v.w);
  }
}

// --------------------------------------------------------- record walk
// One AEAD record (Noise ENCRYPT / DECRYPT, noise.cpp:202-281 semantics).
//   DECRYPT=false: in = plaintext[len]  -> out = ct[len] || tag[16]
//   DECRYPT=true : in = ct[len]||tag    -> the tag is checked over the
//                  ciphertext FIRST (crypto_aead_read, monocypher.c:2912-
//                  2929); only a verified record is decrypted into out.  A
//                  failed one leaves out untouched when in place and zeroes
//                  it when out of place; returns false.  No unauthenticated
//                  plaintext is ever written.
// VEC: in/out are 16-byte aligned and len % 16 == 0 (dwordx4 path).
template <bool DECRYPT, bool VEC>
__device__ __forceinline__ bool aead_record(const uint32_t k[8], uint64_t n,
                                            const uint8_t *in, uint8_t *out,
                                            uint32_t len, const uint8_t *ad,
                                            uint32_t ad_len) {
  const uint32_t n_lo = (uint32_t)n, n_hi = (uint32_t)(n >> 32);
  Poly1305 p;
  {
    uint32_t otk[16];
    chacha20_block(k, 0u, n_lo, n_hi, otk);
    poly_init(p, otk);
  }
  if (ad_len) poly_ad(p, ad, ad_len);
  const uint32_t nfull = len >> 6;
  const uint32_t rem = len & 63u;

  if (DECRYPT) {
    // pass 1: MAC over the ciphertext (reads only)
    for (uint32_t off = 0; off < len; off += 16u) {
      const int nb = (len - off) >= 16u ? 16 : (int)(len - off);
      const uint4 v = load16<VEC>(in + off, nb);
      poly_block(p, v.x, v.y, v.z, v.w);
    }
    poly_block(p, ad_len, 0u, len, 0u);
    uint32_t tag[4];
    poly_final(p, tag);
    const uint4 want = load16<VEC>(in + len, 16);
    const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) |
                          (want.z ^ tag[2]) | (want.w ^ tag[3]);
    if (diff != 0u) {
      // tag mismatch (rare): in place leaves the buffer as it was; a copy
      // gets zeros (no stale bytes of an earlier record)
      if (in != out)
        for (uint32_t off = 0; off < len; off += 16u) {
          const int nb = (len - off) >= 16u ? 16 : (int)(len - off);
          store16<VEC>(out + off, make_uint4(0u, 0u, 0u, 0u), nb);
        }
      return false;
    }
  }
  // (encrypt) or pass 2 (verified decrypt): keystream XOR, encrypt MACs the
  // ciphertext as it goes
  for (uint32_t c = 0; c < nfull; ++c) {
    uint32_t ks[16];
    chacha20_block(k, 1u + c, n_lo, n_hi, ks);
    const uint8_t *src = in + 64u * c;
    uint8_t *dst = out + 64u * c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = load16<VEC>(src + 16 * q, 16);
      uint4 o;
      o.x = v.x ^ ks[4 * q + 0];
      o.y = v.y ^ ks[4 * q + 1];
      o.z = v.z ^ ks[4 * q + 2];
      o.w = v.w ^ ks[4 * q + 3];
      if (!DECRYPT) poly_block(p, o.x, o.y, o.z, o.w);
      store16<VEC>(dst + 16 * q, o, 16);
    }
  }
  if (rem) {
    uint32_t ks[16];
    chacha20_block(k, 1u + nfull, n_lo, n_hi, ks);
    const uint8_t *src = in + 64u * nfull;
    uint8_t *dst = out + 64u * nfull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = (int)rem - 16 * q;
      if (m <= 0) break;
      const int nb = m >= 16 ? 16 : m;
      const uint4 v = load16<VEC>(src + 16 * q, nb);
      // keystream bytes past the record end must not reach the MAC: mask
      const uint4 o = mask_bytes(make_uint4(v.x ^ ks[4 * q + 0], v.y ^ ks[4 * q + 1],
                                            v.z ^ ks[4 * q + 2], v.w ^ ks[4 * q + 3]), nb);
      if (!DECRYPT) poly_block(p, o.x, o.y, o.z, o.w);
      store16<VEC>(dst + 16 * q, o, nb);
    }
  }
  if (!DECRYPT) {
    // length block LE64(ad_len) || LE64(len)
    poly_block(p, ad_len, 0u, len, 0u);
    uint32_t tag[4];
    poly_final(p, tag);
    store16<VEC>(out + len, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
  }
  return true;
}

}  // namespace noise_amd
