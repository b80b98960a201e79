// wave_kernel.hpp -- one wavefront per large record (the "wave" class of
// descriptor batches: 16-byte aligned, AD-free records longer than 16 KiB,
// any length, e.g. the 65519-byte maximum Noise message of BASELINE cfg 4).
//
// The lane-per-record walk would serialise a 64 KiB record on one lane
// (1024 ChaCha blocks) while its 63 neighbours idle; the tile kernel stops
// at 16 KiB.  Here the 64 lanes split ONE record:
//   * lane j owns the contiguous segment of S 64-byte chunks starting at
//     chunk S*j (S = a power of two >= 4 with 64*S*64 >= L), i.e. Sb = 4S
//     Poly1305 blocks, Horner-evaluated with the clamped r;
//   * the segment is processed in R = S/4 rounds of 4 chunks (256 bytes);
//     one round of the whole wave is a 16 KiB window of the record, moved
//     HBM -> LDS by LDS-DMA in 256-byte runs (16 lanes per run, so each
//     wave-instruction touches 4 whole runs), and LDS -> HBM the same way;
//   * recombination: with J the last non-empty lane and n_J its block
//     count, lane j < J multiplies its sum by r^(n_J + Sb*(J-1-j)): one
//     product by r^(n_J) then a 6-level tree over the bits of J-1-j with
//     r^(Sb*2^b); a 64-lane butterfly sums the products.
// Powers: a batch of 16 records shares one key pass (lane l < 16 -> record
// l of the batch: ChaCha block 0, the squaring chain r^(2^b), r^(n_J)),
// parked in LDS (WaveSlot) so the per-record loop carries no power table
// in VGPRs.  Batches are taken from an atomic cursor (records differ in
// size, so static striding would leave tail imbalance).
// Decrypt follows crypto_aead_read (monocypher.c:2912-2929): a MAC pass
// over the ciphertext first, then the ChaCha pass only for a valid tag, so
// an in-place record that fails is left untouched.
// The last partial 16-byte piece (L % 16 != 0) is read whole (a 16-byte
// aligned piece never crosses a page), masked for Poly1305, and written
// byte-wise together with the (then unaligned) tag.
#pragma once
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kWaveBatch = 16;

struct WaveSlot {
  uint32_t k[8];
  uint32_t r[4], s[4];
  uint32_t rn[5];      // r^(n_J), radix 2^26
  uint32_t pw[6][5];   // r^(Sb * 2^b)
  uint32_t tag[4];     // decrypt: the received tag
  uint32_t in_lo, in_hi, out_lo, out_hi;
  uint32_t n_lo, n_hi, len, di;
};

struct WaveGeom {
  uint32_t L, N, Nf, NC, S, log2S, R, J;
};

__device__ __forceinline__ WaveGeom wave_geom(uint32_t L) {
  WaveGeom g;
  g.L = L;
  g.N = (L + 15) / 16;   // Poly1305 data blocks (last may be partial)
  g.Nf = L / 16;         // full 16-byte pieces
  g.NC = (L + 63) / 64;  // ChaCha data blocks
  const uint32_t per = (g.NC + 63) / 64;
  uint32_t l2 = 2;
  while ((1u << l2) < per) ++l2;
  g.log2S = l2;
  g.S = 1u << l2;
  g.R = g.S / 4;
  g.J = (g.N - 1) / (4 * g.S);
  return g;
}

// Poly1305 word mask for the first `rem` (1..15) bytes of a piece
__device__ __forceinline__ uint4 mask_piece(uint4 v, uint32_t rem) {
  uint32_t m[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int b = (int)rem - 4 * w;
    m[w] = b >= 4 ? 0xffffffffu : b <= 0 ? 0u : (1u << (8 * b)) - 1u;
  }
  return make_uint4(v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]);
}

// round k of the current record: physical slot s <- logical piece swz(s)
// = (segment jj, piece p) at byte jj*S*64 + 256k + 16p
__device__ __forceinline__ void wave_dma(lds_u4 *lds3, const uint8_t *src,
                                         const WaveGeom &g, uint32_t k,
                                         uint32_t lane) {
  const uint64_t limit = 16ull * g.N;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t lg = swz(64u * q + lane);
    const uint64_t off = ((uint64_t)(lg >> 4) << (g.log2S + 6)) + 256u * k + 16u * (lg & 15u);
    if (off < limit)
      __builtin_amdgcn_global_load_lds(
          (const void *)(src + off),
          (__attribute__((address_space(3))) void *)(lds3 + 64 * q), 16, 0, 0);
  }
}

__device__ __forceinline__ void poly_select_block(Poly1305 &p, uint4 m, bool take) {
  Poly1305 t = p;
  poly_block(t, m.x, m.y, m.z, m.w);
  p.h0 = take ? t.h0 : p.h0;
  p.h1 = take ? t.h1 : p.h1;
  p.h2 = take ? t.h2 : p.h2;
  p.h3 = take ? t.h3 : p.h3;
  p.h4 = take ? t.h4 : p.h4;
}

// lane sums -> the record's Poly1305 accumulator (all lanes), then the
// length block and the tag
__device__ __forceinline__ void wave_tag(Poly1305 &p, const WaveSlot &ws,
                                         const WaveGeom &g, uint32_t j,
                                         uint32_t tag[4]) {
  F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
  const bool below = j < g.J;
  {
    F26 f;
#pragma unroll
    for (int i = 0; i < 5; ++i) f.a[i] = below ? ws.rn[i] : (i == 0 ? 1u : 0u);
    h = mul26(h, f);
  }
  const uint32_t m = g.J - 1 - j;
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const bool use = below && ((m >> b) & 1u);
    F26 f;
#pragma unroll
    for (int i = 0; i < 5; ++i) f.a[i] = use ? ws.pw[b][i] : (i == 0 ? 1u : 0u);
    h = mul26(h, f);
  }
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    if (b == 4) carry26(h);  // 64 limbs of < 2^26 + 2^9 overflow 32 bits
#pragma unroll
    for (int i = 0; i < 5; ++i) h.a[i] += __shfl_xor(h.a[i], 1 << b);
  }
  carry26(h);
  carry26(h);
  from26(h, p.h0, p.h1, p.h2, p.h3, p.h4);
  poly_block(p, 0u, 0u, g.L, 0u);  // LE64(ad_len = 0) || LE64(L)
  poly_final(p, tag);
}

template <bool DECRYPT>
__global__ __launch_bounds__(64) void k_aead_wave(
    const uint8_t *__restrict__ keys, uint32_t nkeys,
    const noise_gpu_record *__restrict__ recs, const uint32_t *__restrict__ idx,
    const unsigned long long *counts, int cls, unsigned long long *cursor,
    const uint8_t *in, uint8_t *out, uint8_t *status) {
  __shared__ uint4 lds[1024];
  __shared__ WaveSlot slots[kWaveBatch];
  const uint32_t lane = threadIdx.x;
  uint64_t base = 0;
  for (int c = 0; c < cls; ++c) base += counts[c];
  const uint64_t count = counts[cls];

#pragma unroll 1
  for (;;) {
    uint64_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(cursor, (unsigned long long)kWaveBatch);
    b0 = join64(uniform32((uint32_t)(b0 >> 32)), uniform32((uint32_t)b0));  // lane 0's claim
    if (b0 >= count) break;
    const uint32_t nb = (count - b0) < (uint64_t)kWaveBatch ? (uint32_t)(count - b0) : kWaveBatch;

    // ---- key pass: lane l < nb -> record b0 + l ---------------------------
    if (lane < nb) {
      WaveSlot &ws = slots[lane];
      const uint32_t di = idx[base + b0 + lane];
      const noise_gpu_record d = recs[di];
      const uint32_t ki = d.key_idx < nkeys ? d.key_idx : 0u;  // classifier checked
      const u32x4 *kp = reinterpret_cast<const u32x4 *>(keys + 32ull * ki);
      const u32x4 ka = kp[0], kb = kp[1];
      uint32_t k8[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
      uint32_t otk[16];
      chacha20_block(k8, 0u, (uint32_t)d.nonce, (uint32_t)(d.nonce >> 32), otk);
#pragma unroll
      for (int i = 0; i < 8; ++i) ws.k[i] = k8[i];
      ws.r[0] = otk[0] & 0x0fffffffu;
      ws.r[1] = otk[1] & 0x0ffffffcu;
      ws.r[2] = otk[2] & 0x0ffffffcu;
      ws.r[3] = otk[3] & 0x0ffffffcu;
      ws.s[0] = otk[4]; ws.s[1] = otk[5]; ws.s[2] = otk[6]; ws.s[3] = otk[7];
      const WaveGeom g = wave_geom(d.len);
      const uint32_t log2Sb = g.log2S + 2;
      const uint32_t nJ = g.N - (g.J << log2Sb);  // 1 .. Sb
      F26 x = to26(ws.r[0], ws.r[1], ws.r[2], ws.r[3], 0u);
      F26 rn;
      rn.a[0] = 1u; rn.a[1] = rn.a[2] = rn.a[3] = rn.a[4] = 0u;
#pragma unroll 1
      for (uint32_t b = 0; b <= log2Sb + 5; ++b) {
        if (b > 0) x = mul26(x, x);  // r^(2^b)
        if ((nJ >> b) & 1u) rn = mul26(rn, x);
        if (b >= log2Sb) {
#pragma unroll
          for (int i = 0; i < 5; ++i) ws.pw[b - log2Sb][i] = x.a[i];
        }
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) ws.rn[i] = rn.a[i];
      if (DECRYPT) {
        const uint8_t *tp = in + d.in_off + d.len;
#pragma unroll
        for (int w = 0; w < 4; ++w) ws.tag[w] = ld_bytes(tp + 4 * w, 4);
      }
      ws.in_lo = (uint32_t)d.in_off; ws.in_hi = (uint32_t)(d.in_off >> 32);
      ws.out_lo = (uint32_t)d.out_off; ws.out_hi = (uint32_t)(d.out_off >> 32);
      ws.n_lo = (uint32_t)d.nonce; ws.n_hi = (uint32_t)(d.nonce >> 32);
      ws.len = d.len;
      ws.di = di;
    }
    wait_all();
    wave_lds_fence();

#pragma unroll 1
    for (uint32_t t = 0; t < nb; ++t) {
      const WaveSlot &ws = slots[t];
      const WaveGeom g = wave_geom(uniform32(ws.len));
      const uint8_t *src = in + join64(uniform32(ws.in_hi), uniform32(ws.in_lo));
      uint8_t *dst = out + join64(uniform32(ws.out_hi), uniform32(ws.out_lo));
      const uint32_t n_lo = uniform32(ws.n_lo);
      const uint32_t n_hi = uniform32(ws.n_hi);
      const uint32_t j = lane;
      const uint32_t rem = g.L - 16u * g.Nf;  // bytes of the partial piece
      const uint32_t b_seg = j << (g.log2S + 2);           // ... in Poly blocks

      Poly1305 p;
      p.r0 = ws.r[0]; p.r1 = ws.r[1]; p.r2 = ws.r[2]; p.r3 = ws.r[3];
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      p.s0 = ws.s[0]; p.s1 = ws.s[1]; p.s2 = ws.s[2]; p.s3 = ws.s[3];
      p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
      uint4 stash = make_uint4(0u, 0u, 0u, 0u);  // the partial piece, if mine

      bool ok = true;
      if (DECRYPT) {
        // ---- MAC pass over the ciphertext --------------------------------
        wave_dma(NOISE_LDS3(lds), src, g, 0, lane);
#pragma unroll 1
        for (uint32_t k = 0; k < g.R; ++k) {
          wait_vmem();
          wave_lds_fence();
          uint4 v[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = lds[swz(16u * j + q)];
          wait_lds();
          wave_lds_fence();
          if (k + 1 < g.R) wave_dma(NOISE_LDS3(lds), src, g, k + 1, lane);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t b = b_seg + 16u * k + q;
            poly_select_block(p, v[q], b < g.Nf);
            if (b == g.Nf) stash = v[q];
          }
        }
        poly_select_block(p, mask_piece(stash, rem),
                          rem != 0 && g.Nf >= b_seg && g.Nf < b_seg + 4 * g.S);
        uint32_t tag[4];
        wave_tag(p, ws, g, j, tag);
        const uint32_t diff = (tag[0] ^ ws.tag[0]) | (tag[1] ^ ws.tag[1]) |
                              (tag[2] ^ ws.tag[2]) | (tag[3] ^ ws.tag[3]);
        ok = diff == 0u;
        if (lane == 0) status[ws.di] = ok ? 0u : 1u;
        if (!ok) {
          if (src != dst) {  // zero a copy; an in-place record stays as it was
            for (uint64_t off = 16ull * lane; off < 16ull * g.Nf; off += 1024)
              store16<true>(dst + off, make_uint4(0u, 0u, 0u, 0u), 16);
            if (lane == 0)
              for (uint32_t i = 16u * g.Nf; i < g.L; ++i) dst[i] = 0;
          }
          continue;
        }
      }

      // ---- ChaCha pass (encrypt: + MAC over the ciphertext) ---------------
      uint32_t kt[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) kt[i] = uniform32(ws.k[i]);
      const ChaPre pre = chacha_pre(kt, n_lo, n_hi);
      wave_dma(NOISE_LDS3(lds), src, g, 0, lane);
#pragma unroll 1
      for (uint32_t k = 0; k < g.R; ++k) {
        wait_vmem();
        wave_lds_fence();
        const uint32_t c0 = (j << g.log2S) + 4u * k;  // first chunk this round
        uint32_t ks[16];
        chacha20_block_pre(kt, 1u + c0, pre, n_lo, n_hi, ks);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          uint32_t ksn[16];
          if (kk + 1 < 4) chacha20_block_pre(kt, 2u + c0 + kk, pre, n_lo, n_hi, ksn);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t slot = swz(16u * j + 4u * kk + q);
            const uint4 v = lds[slot];
            uint4 o;
            o.x = v.x ^ ks[4 * q + 0];
            o.y = v.y ^ ks[4 * q + 1];
            o.z = v.z ^ ks[4 * q + 2];
            o.w = v.w ^ ks[4 * q + 3];
            lds[slot] = o;
            const uint32_t b = b_seg + 16u * k + 4u * kk + q;
            if (!DECRYPT) poly_select_block(p, o, b < g.Nf);
            if (b == g.Nf) stash = o;
          }
          if (kk + 1 < 4) {
#pragma unroll
            for (int i = 0; i < 16; ++i) ks[i] = ksn[i];
          }
        }
        wait_lds();
        wave_lds_fence();
        uint4 ov[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) ov[q] = lds[64 * q + lane];
        wait_lds();
        wave_lds_fence();
        if (k + 1 < g.R) wave_dma(NOISE_LDS3(lds), src, g, k + 1, lane);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const uint32_t lg = swz(64u * q + lane);
          const uint64_t off = ((uint64_t)(lg >> 4) << (g.log2S + 6)) + 256u * k + 16u * (lg & 15u);
          if (off + 16 <= g.L) store16<true>(dst + off, ov[q], 16);
        }
      }
      const bool has_partial = rem != 0 && g.Nf >= b_seg && g.Nf < b_seg + 4 * g.S;
      uint32_t tag[4];
      if (!DECRYPT) {
        poly_select_block(p, mask_piece(stash, rem), has_partial);
        wave_tag(p, ws, g, j, tag);
      }
      // tail: the partial piece (byte-wise) and, for encrypt, the tag
      if (j == g.J) {
        if (rem != 0) {
          const uint32_t w4[4] = {stash.x, stash.y, stash.z, stash.w};
          for (uint32_t i = 0; i < rem; ++i)
            dst[16u * g.Nf + i] = (uint8_t)(w4[i >> 2] >> (8 * (i & 3)));
        }
        if (!DECRYPT) {
          if (rem == 0) {
            store16<true>(dst + g.L, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
          } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) st_bytes(dst + g.L + 4 * w, tag[w], 4);
          }
        }
      }
    }
    // every lane is done with this batch's slots before the next key pass
    wait_all();
    wave_lds_fence();
  }
}

}  // namespace noise_amd
