// x25519_device.hpp -- X25519 (RFC 7748 §5) as a per-lane device function:
// field arithmetic mod 2^255-19 in ten 26/25-bit limbs (radix 2^25.5) in
// VGPRs and the constant-time Montgomery ladder.  Shared by the batched
// X25519 kernel (x25519_kernels.hip) and the batched handshake kernels
// (handshake_kernels.hip).  Replaces monocypher.c:1487-1563 (scalarmult,
// crypto_x25519) as called by noise.cpp:164-177.
//
// A field product is 100 32x32->64 multiply-adds (v_mad_u64_u32) plus one
// carry pass (a square: 55); sums and differences stay uncarried into the
// next product.  The ladder has no secret-dependent branch or address: the
// swap is an arithmetic mask, so all 64 lanes of a wave run the same
// instruction stream (constant time per lane, no divergence).  Inversion by
// the standard 254-squaring / 11-multiplication chain for p-2.
//
// Formula source: fe_mul / fe_sq below are the public-domain ref10 schoolbook
// products in radix 2^25.5 (SUPERCOP crypto_scalarmult/curve25519/ref10,
// fe_mul.c / fe_sq.c), the same formulas monocypher.c:1225-1325 carries; the
// term order and the 19*g / 2*f temporaries follow them.  The carry handling
// (unsigned, uncarried sums fed to the next product, one carry pass per
// product) is this file's own.
#pragma once
#include "chachapoly_device.hpp"

namespace noise_amd {
namespace x25519 {
constexpr uint32_t kM26 = (1u << 26) - 1, kM25 = (1u << 25) - 1;

struct Fe {
  uint32_t v[10];
};

__device__ __forceinline__ void fe_carry(Fe &h, uint64_t t[10]) {
  // t: 64-bit column sums -> h: carried limbs (< 2^26 / 2^25, h1 slightly more)
  uint64_t c;
  c = t[0] >> 26; t[1] += c; t[0] &= kM26;
  c = t[1] >> 25; t[2] += c; t[1] &= kM25;
  c = t[2] >> 26; t[3] += c; t[2] &= kM26;
  c = t[3] >> 25; t[4] += c; t[3] &= kM25;
  c = t[4] >> 26; t[5] += c; t[4] &= kM26;
  c = t[5] >> 25; t[6] += c; t[5] &= kM25;
  c = t[6] >> 26; t[7] += c; t[6] &= kM26;
  c = t[7] >> 25; t[8] += c; t[7] &= kM25;
  c = t[8] >> 26; t[9] += c; t[8] &= kM26;
  c = t[9] >> 25; t[9] &= kM25; t[0] += 19 * c;
  c = t[0] >> 26; t[0] &= kM26; t[1] += c;
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = (uint32_t)t[i];
}

__device__ __forceinline__ void fe_reduce(Fe &h) {
  uint64_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = h.v[i];
  fe_carry(h, t);
}

// Sums and differences are NOT carried: every operand of the ladder's adds
// and subs is a carried product (limbs <= 2^26 / 2^25 + small), so their
// results stay below 2^27.6 per limb, and fe_mul / fe_sq accept that (19 * limb
// < 2^32, every 64-bit column sum < 2^63.7).
__device__ __forceinline__ void fe_add(Fe &h, const Fe &f, const Fe &g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// f + 2p - g (g carried: limbs <= 2^26 / 2^25 + small)
__device__ __forceinline__ void fe_sub(Fe &h, const Fe &f, const Fe &g) {
  h.v[0] = f.v[0] + 0x7ffffdau - g.v[0];  // 2^27 - 38
#pragma unroll
  for (int i = 1; i < 10; ++i)
    h.v[i] = f.v[i] + ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - g.v[i];  // 2^26-2 / 2^27-2
}

__device__ __forceinline__ uint64_t m64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

__device__ __forceinline__ void fe_mul(Fe &h, const Fe &F, const Fe &G) {
  const uint32_t *f = F.v, *g = G.v;
  const uint32_t g1 = 19 * g[1], g2 = 19 * g[2], g3 = 19 * g[3], g4 = 19 * g[4], g5 = 19 * g[5],
                 g6 = 19 * g[6], g7 = 19 * g[7], g8 = 19 * g[8], g9 = 19 * g[9];
  const uint32_t f1 = 2 * f[1], f3 = 2 * f[3], f5 = 2 * f[5], f7 = 2 * f[7], f9 = 2 * f[9];
  uint64_t t[10];
  t[0] = m64(f[0], g[0]) + m64(f1, g9) + m64(f[2], g8) + m64(f3, g7) + m64(f[4], g6) +
         m64(f5, g5) + m64(f[6], g4) + m64(f7, g3) + m64(f[8], g2) + m64(f9, g1);
  t[1] = m64(f[0], g[1]) + m64(f[1], g[0]) + m64(f[2], g9) + m64(f[3], g8) + m64(f[4], g7) +
         m64(f[5], g6) + m64(f[6], g5) + m64(f[7], g4) + m64(f[8], g3) + m64(f[9], g2);
  t[2] = m64(f[0], g[2]) + m64(f1, g[1]) + m64(f[2], g[0]) + m64(f3, g9) + m64(f[4], g8) +
         m64(f5, g7) + m64(f[6], g6) + m64(f7, g5) + m64(f[8], g4) + m64(f9, g3);
  t[3] = m64(f[0], g[3]) + m64(f[1], g[2]) + m64(f[2], g[1]) + m64(f[3], g[0]) + m64(f[4], g9) +
         m64(f[5], g8) + m64(f[6], g7) + m64(f[7], g6) + m64(f[8], g5) + m64(f[9], g4);
  t[4] = m64(f[0], g[4]) + m64(f1, g[3]) + m64(f[2], g[2]) + m64(f3, g[1]) + m64(f[4], g[0]) +
         m64(f5, g9) + m64(f[6], g8) + m64(f7, g7) + m64(f[8], g6) + m64(f9, g5);
  t[5] = m64(f[0], g[5]) + m64(f[1], g[4]) + m64(f[2], g[3]) + m64(f[3], g[2]) + m64(f[4], g[1]) +
         m64(f[5], g[0]) + m64(f[6], g9) + m64(f[7], g8) + m64(f[8], g7) + m64(f[9], g6);
  t[6] = m64(f[0], g[6]) + m64(f1, g[5]) + m64(f[2], g[4]) + m64(f3, g[3]) + m64(f[4], g[2]) +
         m64(f5, g[1]) + m64(f[6], g[0]) + m64(f7, g9) + m64(f[8], g8) + m64(f9, g7);
  t[7] = m64(f[0], g[7]) + m64(f[1], g[6]) + m64(f[2], g[5]) + m64(f[3], g[4]) + m64(f[4], g[3]) +
         m64(f[5], g[2]) + m64(f[6], g[1]) + m64(f[7], g[0]) + m64(f[8], g9) + m64(f[9], g8);
  t[8] = m64(f[0], g[8]) + m64(f1, g[7]) + m64(f[2], g[6]) + m64(f3, g[5]) + m64(f[4], g[4]) +
         m64(f5, g[3]) + m64(f[6], g[2]) + m64(f7, g[1]) + m64(f[8], g[0]) + m64(f9, g9);
  t[9] = m64(f[0], g[9]) + m64(f[1], g[8]) + m64(f[2], g[7]) + m64(f[3], g[6]) + m64(f[4], g[5]) +
         m64(f[5], g[4]) + m64(f[6], g[3]) + m64(f[7], g[2]) + m64(f[8], g[1]) + m64(f[9], g[0]);
  fe_carry(h, t);
}

// f^2 with the symmetric products merged: 55 multiply-adds instead of 100
__device__ __forceinline__ void fe_sq(Fe &h, const Fe &F) {
  const uint32_t *f = F.v;
  const uint32_t f0_2 = 2 * f[0], f1_2 = 2 * f[1], f2_2 = 2 * f[2], f3_2 = 2 * f[3],
                 f4_2 = 2 * f[4], f5_2 = 2 * f[5], f6_2 = 2 * f[6], f7_2 = 2 * f[7];
  const uint32_t f5_38 = 38 * f[5], f6_19 = 19 * f[6], f7_38 = 38 * f[7], f8_19 = 19 * f[8],
                 f9_38 = 38 * f[9];
  uint64_t t[10];
  t[0] = m64(f[0], f[0]) + m64(f1_2, f9_38) + m64(f2_2, f8_19) + m64(f3_2, f7_38) +
         m64(f4_2, f6_19) + m64(f[5], f5_38);
  t[1] = m64(f0_2, f[1]) + m64(f[2], f9_38) + m64(f3_2, f8_19) + m64(f[4], f7_38) +
         m64(f5_2, f6_19);
  t[2] = m64(f0_2, f[2]) + m64(f1_2, f[1]) + m64(f3_2, f9_38) + m64(f4_2, f8_19) +
         m64(f5_2, f7_38) + m64(f[6], f6_19);
  t[3] = m64(f0_2, f[3]) + m64(f1_2, f[2]) + m64(f[4], f9_38) + m64(f5_2, f8_19) +
         m64(f[6], f7_38);
  t[4] = m64(f0_2, f[4]) + m64(f1_2, f3_2) + m64(f[2], f[2]) + m64(f5_2, f9_38) +
         m64(f6_2, f8_19) + m64(f[7], f7_38);
  t[5] = m64(f0_2, f[5]) + m64(f1_2, f[4]) + m64(f2_2, f[3]) + m64(f[6], f9_38) +
         m64(f7_2, f8_19);
  t[6] = m64(f0_2, f[6]) + m64(f1_2, f5_2) + m64(f2_2, f[4]) + m64(f3_2, f[3]) +
         m64(f7_2, f9_38) + m64(f[8], f8_19);
  t[7] = m64(f0_2, f[7]) + m64(f1_2, f[6]) + m64(f2_2, f[5]) + m64(f3_2, f[4]) +
         m64(f[8], f9_38);
  t[8] = m64(f0_2, f[8]) + m64(f1_2, f7_2) + m64(f2_2, f[6]) + m64(f3_2, f5_2) +
         m64(f[4], f[4]) + m64(f[9], f9_38);
  t[9] = m64(f0_2, f[9]) + m64(f1_2, f[8]) + m64(f2_2, f[7]) + m64(f3_2, f[6]) +
         m64(f4_2, f[5]);
  fe_carry(h, t);
}

__device__ __forceinline__ void fe_sqn(Fe &h, const Fe &f, int n) {
  fe_sq(h, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

__device__ __forceinline__ void fe_mul121665(Fe &h, const Fe &f) {
  uint64_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = m64(f.v[i], 121665u);
  fe_carry(h, t);
}

// z^(p-2) = z^(2^255 - 21)
__device__ __forceinline__ void fe_invert(Fe &out, const Fe &z) {
  Fe t0, t1, t2, t3;
  fe_sq(t0, z);           // 2
  fe_sqn(t1, t0, 2);      // 8
  fe_mul(t1, z, t1);      // 9
  fe_mul(t0, t0, t1);     // 11
  fe_sq(t2, t0);          // 22
  fe_mul(t1, t1, t2);     // 2^5 - 1
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);     // 2^10 - 1
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);     // 2^20 - 1
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);     // 2^40 - 1
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);     // 2^50 - 1
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);     // 2^100 - 1
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);     // 2^200 - 1
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);     // 2^250 - 1
  fe_sqn(t1, t1, 5);      // 2^255 - 32
  fe_mul(out, t1, t0);    // 2^255 - 21
}

__device__ __forceinline__ void fe_frombytes(Fe &h, const uint32_t w[8]) {
  // bit offsets of the limbs: 0 26 51 77 102 128 153 179 204 230
  auto bits = [&](int off, int n) -> uint32_t {
    const int wi = off >> 5, sh = off & 31;
    uint64_t x = w[wi] >> sh;
    if (sh + n > 32 && wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    return (uint32_t)x & ((1u << n) - 1u);
  };
  h.v[0] = bits(0, 26);   h.v[1] = bits(26, 25);
  h.v[2] = bits(51, 26);  h.v[3] = bits(77, 25);
  h.v[4] = bits(102, 26); h.v[5] = bits(128, 25);
  h.v[6] = bits(153, 26); h.v[7] = bits(179, 25);
  h.v[8] = bits(204, 26); h.v[9] = bits(230, 25);  // bit 255 ignored (RFC 7748 §5)
}

__device__ __forceinline__ void fe_tobytes(uint32_t w[8], const Fe &f) {
  Fe h = f;
  fe_reduce(h);
  fe_reduce(h);
  // q = 1 iff h >= p, by the carry of h + 19 through all limbs
  uint32_t q = (h.v[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (h.v[i] + q) >> ((i & 1) ? 25 : 26);
  h.v[0] += 19 * q;
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = (i & 1) ? 25 : 26;
    c = h.v[i] >> b;
    h.v[i] &= (1u << b) - 1u;
    h.v[i + 1] += c;
  }
  h.v[9] &= kM25;
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    acc |= (uint64_t)h.v[i] << nb;
    nb += (i & 1) ? 25 : 26;
    while (nb >= 32) {
      w[wi++] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
    }
  }
  w[7] = (uint32_t)acc;  // the last 31 bits (255 in all)
}

__device__ __forceinline__ void fe_cswap(Fe &a, Fe &b, uint32_t swap) {
  const uint32_t mask = 0u - swap;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t t = mask & (a.v[i] ^ b.v[i]);
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}

// out = X25519(k, u): k clamped here (RFC 7748 §5), u's bit 255 ignored
__device__ __forceinline__ void scalarmult(uint32_t out[8], const uint32_t kin[8],
                                           const uint32_t u[8]) {
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = kin[j];
  k[0] &= ~7u;                                   // clamp: clear bits 0-2,
  k[7] = (k[7] & 0x7fffffffu) | 0x40000000u;     // clear 255, set 254
  Fe x1, x2, z2, x3, z3;
  fe_frombytes(x1, u);
  x3 = x1;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    x2.v[j] = j == 0 ? 1u : 0u;
    z2.v[j] = 0u;
    z3.v[j] = j == 0 ? 1u : 0u;
  }
  uint32_t swap = 0;
  Fe a, aa, b, bb, e, c, d, da, cb, t;
#pragma unroll 1
  for (int pos = 254; pos >= 0; --pos) {
    const uint32_t bit = (k[pos >> 5] >> (pos & 31)) & 1u;
    swap ^= bit;
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    swap = bit;
    fe_add(a, x2, z2);
    fe_sq(aa, a);
    fe_sub(b, x2, z2);
    fe_sq(bb, b);
    fe_sub(e, aa, bb);
    fe_add(c, x3, z3);
    fe_sub(d, x3, z3);
    fe_mul(da, d, a);
    fe_mul(cb, c, b);
    fe_add(t, da, cb);
    fe_sq(x3, t);
    fe_sub(t, da, cb);
    fe_sq(t, t);
    fe_mul(z3, x1, t);
    fe_mul(x2, aa, bb);
    fe_mul121665(t, e);
    fe_add(t, aa, t);
    fe_mul(z2, e, t);
  }
  fe_cswap(x2, x3, swap);
  fe_cswap(z2, z3, swap);
  fe_invert(z2, z2);
  fe_mul(x2, x2, z2);
  fe_tobytes(out, x2);
}

// ---- fixed base: public keys X25519(k, 9) --------------------------------
// [k]B on edwards25519 (the birational image of u = 9), then u = (Z+Y)/(Z-Y)
// (RFC 7748 §4.1).  k is recoded into 64 signed radix-16 digits
// d_i = n_i + b_(4i-1) - 16 b_(4i+3) in [-8, 8] (Booth: each digit from five
// scalar bits, no carry chain), and [k]B = sum_i d_i 16^i B: 64 mixed
// additions of table points kBaseTable[i][|d_i|-1] = |d_i| 16^i B (affine
// niels form (y+x, y-x, 2dxy), tools/gen_base_table.py).  Constant time per
// lane: every window reads all 8 entries of its row (the row index i is
// public and wave-uniform, so they are scalar loads) and keeps the wanted one
// with masks; a negative digit swaps y+x / y-x and negates 2dxy with masks.
// ~2.9x fewer VALU instructions than the ladder with u = 9.
static __constant__ const uint32_t kBaseTable[64][8][3][10] = {
#include "ed25519_base_table.inc"
};

struct Niels {
  Fe yp, ym, xy2d;
};
struct P3 {
  Fe X, Y, Z, T;
};

__device__ __forceinline__ void fe_zero(Fe &h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0u;
}
__device__ __forceinline__ void fe_one(Fe &h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = i == 0 ? 1u : 0u;
}
__device__ __forceinline__ void fe_cmov(Fe &t, const Fe &e, uint32_t mask) {
#pragma unroll
  for (int i = 0; i < 10; ++i) t.v[i] ^= mask & (t.v[i] ^ e.v[i]);
}

// t = d * 16^i * B in niels form, d in [-8, 8] (secret), row i public
__device__ __forceinline__ void base_select(Niels &t, int i, int32_t d) {
  const uint32_t neg = (uint32_t)d >> 31;
  const uint32_t mag = (uint32_t)((d ^ -(int32_t)neg) + (int32_t)neg);  // |d|
  fe_one(t.yp);
  fe_one(t.ym);
  fe_zero(t.xy2d);
#pragma unroll 1
  for (int j = 0; j < 8; ++j) {
    const uint32_t m = 0u - (uint32_t)(mag == (uint32_t)(j + 1));
    const uint32_t *e = kBaseTable[i][j][0];
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      t.yp.v[l] ^= m & (t.yp.v[l] ^ e[l]);
      t.ym.v[l] ^= m & (t.ym.v[l] ^ e[10 + l]);
      t.xy2d.v[l] ^= m & (t.xy2d.v[l] ^ e[20 + l]);
    }
  }
  // -(x, y) = (-x, y): swap y+x and y-x, negate 2dxy
  const uint32_t nm = 0u - neg;
  Fe sw = t.yp, mx, z;
  fe_cmov(t.yp, t.ym, nm);
  fe_cmov(t.ym, sw, nm);
  fe_zero(z);
  fe_sub(mx, z, t.xy2d);  // 2p - 2dxy
  fe_cmov(t.xy2d, mx, nm);
}

// h <- h + q (extended + affine niels: 7 multiplications).  Inputs carried;
// every difference below has a carried subtrahend, every product input
// stays < 2^27.7 per limb (fe_mul's bound).
__device__ __forceinline__ void ge_madd(P3 &h, const Niels &q) {
  Fe a, b, A, Bm, C, D, X1, Y1, Z1, T1;
  fe_add(a, h.Y, h.X);
  fe_sub(b, h.Y, h.X);
  fe_mul(A, a, q.yp);
  fe_mul(Bm, b, q.ym);
  fe_mul(C, q.xy2d, h.T);
  fe_add(D, h.Z, h.Z);
  fe_reduce(D);
  fe_sub(X1, A, Bm);
  fe_add(Y1, A, Bm);
  fe_add(Z1, D, C);
  fe_sub(T1, D, C);
  fe_mul(h.X, X1, T1);
  fe_mul(h.Y, Y1, Z1);
  fe_mul(h.Z, Z1, T1);
  fe_mul(h.T, X1, Y1);
}

__device__ __forceinline__ void base_scalarmult(uint32_t out[8], const uint32_t kin[8]) {
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = kin[j];
  k[0] &= ~7u;                                   // clamp (RFC 7748 §5)
  k[7] = (k[7] & 0x7fffffffu) | 0x40000000u;
  P3 h;  // identity (0 : 1 : 1 : 0)
  fe_zero(h.X);
  fe_one(h.Y);
  fe_one(h.Z);
  fe_zero(h.T);
  uint32_t carry = 0;  // b_(4i-1)
#pragma unroll 1
  for (int i = 0; i < 64; ++i) {
    uint32_t w;
    switch (i >> 3) {  // wave-uniform
      case 0: w = k[0]; break;
      case 1: w = k[1]; break;
      case 2: w = k[2]; break;
      case 3: w = k[3]; break;
      case 4: w = k[4]; break;
      case 5: w = k[5]; break;
      case 6: w = k[6]; break;
      default: w = k[7]; break;
    }
    const uint32_t nib = (w >> (4 * (i & 7))) & 15u;
    const uint32_t top = nib >> 3;
    const int32_t d = (int32_t)(nib + carry) - (int32_t)(top << 4);
    carry = top;
    Niels t;
    base_select(t, i, d);
    ge_madd(h, t);
  }
  // bit 255 is clear after clamping: no final carry.  u = (Z + Y) / (Z - Y)
  Fe num, den, u;
  fe_add(num, h.Z, h.Y);
  fe_sub(den, h.Z, h.Y);
  fe_invert(den, den);
  fe_mul(u, num, den);
  fe_tobytes(out, u);
}

}  // namespace x25519
}  // namespace noise_amd
