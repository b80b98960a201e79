// rec32_kernel.hpp -- descriptor records of exactly 32 KiB, one wave per
// record, the whole record resident in two 16 KiB LDS windows
// (records_kernels.hip, round 5).
//
// Decrypt checks a record's tag before any of its plaintext is stored
// (crypto_aead_read, monocypher.c:2912-2929).  Here the wave holds the whole
// record, so it reads the ciphertext once: Poly1305 over both windows, the
// tag, then the keystream and the stores.  Lane j owns the contiguous span
// [512 j, 512 j + 512): window k holds bytes [512 j + 256 k, +256) of every
// span (piece i of lane j at slot 16 j + (i ^ (j & 15)): the owner's
// ds_read_b128 are conflict-free).  Memory instruction q (LDS-DMA in, store
// out) moves the 256-byte chunks of spans 4q .. 4q + 3, 16 lanes each.  The
// next record's window k is loaded as soon as this record's window k is
// stored, so its DMA runs under the rest of this record.  A super-tile is 8
// records: lanes 0..7 compute their one-time keys and r^(32 2^b) once.
#pragma once
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kRec32RPS = 8;  // records per super-tile

template <bool DECRYPT>
__global__ __launch_bounds__(64) void k_rec32(const TileArgs a) {
  __shared__ uint4 win[2][16 * 64];        // the record: two windows of 16 KiB
  __shared__ uint32_t kp[kRec32RPS][40];   // r[4], s[4], r^(32 2^b) [6][5]
  constexpr uint32_t L = 32768u, S = 512u;
  const uint32_t lane = threadIdx.x, sw = lane & 15u;
  const uint64_t base = a.cls_base[a.cls], n = a.counts[a.cls];

  // record byte of lane's piece in memory instruction q of window k
  auto moff = [&](int q, uint32_t k) -> uint32_t {
    const uint32_t jq = 4u * (uint32_t)q + (lane >> 4);
    return jq * S + 256u * k + 16u * ((lane & 15u) ^ (jq & 15u));
  };
  auto load_win = [&](const uint8_t *rin, uint32_t k) {
#pragma unroll
    for (int q = 0; q < 16; ++q)
      lds_dma16_v<true>(rin + moff(q, k), (lds_void *)NOISE_LDS3(&win[k][64 * q]));
  };
  auto store_win = [&](uint8_t *rout, uint32_t k, bool zero) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint4 v = zero ? make_uint4(0u, 0u, 0u, 0u) : win[k][64u * q + lane];
      store16<true>(rout + moff(q, k), v, 16);
    }
  };

#pragma unroll 1
  for (uint64_t super0 = (uint64_t)blockIdx.x * kRec32RPS; super0 < n;
       super0 += (uint64_t)gridDim.x * kRec32RPS) {
    // ---- key pass: lane l < kRec32RPS -> record super0 + l ----------------
    uint32_t own_di = 0, own_k[8];
    uint64_t own_n = 0, own_in = 0, own_out = 0;
    {
      const uint64_t rec = super0 + lane;
      uint32_t ki = 0;
      if (lane < (uint32_t)kRec32RPS && rec < n) {
        own_di = a.idx[base + rec];
        const noise_gpu_record d = a.recs[own_di];
        ki = d.key_idx < a.nkeys ? d.key_idx : 0u;  // (the classifier routed bad rows away)
        own_n = d.nonce;
        own_in = d.in_off;
        own_out = d.out_off;
      }
      const u32x4 *kp4 = reinterpret_cast<const u32x4 *>(a.keys + 32ull * ki);
      const u32x4 ka = kp4[0], kb = kp4[1];
      own_k[0] = ka.x; own_k[1] = ka.y; own_k[2] = ka.z; own_k[3] = ka.w;
      own_k[4] = kb.x; own_k[5] = kb.y; own_k[6] = kb.z; own_k[7] = kb.w;
      uint32_t otk[16];
      chacha20_block(own_k, 0u, (uint32_t)own_n, (uint32_t)(own_n >> 32), otk);
      if (lane < (uint32_t)kRec32RPS) {
        const uint32_t r0 = otk[0] & 0x0fffffffu, r1 = otk[1] & 0x0ffffffcu,
                       r2 = otk[2] & 0x0ffffffcu, r3 = otk[3] & 0x0ffffffcu;
        uint32_t *K = kp[lane];
        K[0] = r0; K[1] = r1; K[2] = r2; K[3] = r3;
        K[4] = otk[4]; K[5] = otk[5]; K[6] = otk[6]; K[7] = otk[7];
        F26 y = to26(r0, r1, r2, r3, 0u);
#pragma unroll
        for (int b = 0; b < 5; ++b) y = mul26(y, y);  // r^32 (a span's 32 blocks)
#pragma unroll
        for (int b = 0; b < 6; ++b) {
#pragma unroll
          for (int i = 0; i < 5; ++i) K[8 + 5 * b + i] = y.a[i];
          if (b < 5) y = mul26(y, y);
        }
      }
    }
    // the first record's windows
    const uint32_t nrec = (uint32_t)(n - super0 < (uint64_t)kRec32RPS ? n - super0 : kRec32RPS);
    {
      const uint64_t in0 = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_in >> 32), 0),
                                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_in, 0));
      load_win(a.in + in0, 0u);
      load_win(a.in + in0, 1u);
    }
    wait_lds();
    wave_lds_fence();

#pragma unroll 1
    for (uint32_t i = 0; i < nrec; ++i) {
      const uint32_t di = (uint32_t)__builtin_amdgcn_readlane((int)own_di, (int)i);
      const uint64_t in_off = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_in >> 32), (int)i),
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_in, (int)i));
      const uint64_t out_off = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_out >> 32), (int)i),
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_out, (int)i));
      const uint32_t n_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_n, (int)i);
      const uint32_t n_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_n >> 32), (int)i);
      uint32_t kt[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) kt[w] = (uint32_t)__builtin_amdgcn_readlane((int)own_k[w], (int)i);
      const uint32_t *K = kp[i];
      const uint8_t *rin = a.in + in_off;
      uint8_t *rout = a.out + out_off;
      // the next record's input (its windows go out as this one's are stored)
      const bool has_next = i + 1u < nrec;
      const uint32_t ni = has_next ? i + 1u : i;
      const uint64_t nin = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_in >> 32), (int)ni),
                                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_in, (int)ni));
      Poly1305 p;
      p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
      p.r0 = K[0]; p.r1 = K[1]; p.r2 = K[2]; p.r3 = K[3];
      p.rr0 = (p.r0 >> 2) * 5u;
      p.rr1 = p.r1 + (p.r1 >> 2);
      p.rr2 = p.r2 + (p.r2 >> 2);
      p.rr3 = p.r3 + (p.r3 >> 2);
      p.r0lo = p.r0 & 3u;
      const ChaPre pre = chacha_pre(kt, n_lo, n_hi);
      // window k's keystream over my span's pieces, in LDS; encrypt: Poly1305
      // of the ciphertext as it goes
      auto xor_win = [&](uint32_t k) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint32_t ks[16];
          chacha20_block_pre(kt, 1u + ((lane * S + 256u * k + 64u * c) >> 6), pre, n_lo, n_hi, ks);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const uint32_t slot = 16u * lane + ((4u * c + qq) ^ sw);
            const uint4 v = win[k][slot];
            const uint4 o = make_uint4(v.x ^ ks[4 * qq + 0], v.y ^ ks[4 * qq + 1], v.z ^ ks[4 * qq + 2],
                                       v.w ^ ks[4 * qq + 3]);
            if (!DECRYPT) poly_block(p, o.x, o.y, o.z, o.w);
            win[k][slot] = o;
          }
        }
      };
      wait_vmem();  // this record's windows (and the last record's stores)
      wave_lds_fence();
      bool ok = true;
      if (DECRYPT) {
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint4 v = win[k][16u * lane + ((uint32_t)q ^ sw)];
            poly_block(p, v.x, v.y, v.z, v.w);
          }
        }
      } else {
        xor_win(0u);
        xor_win(1u);
      }
      // ---- the tag: sum_j H_j r^(32 (63 - j)) + the length block ---------
      uint32_t tag[4];
      {
        F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
        const uint32_t m = 63u - lane;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          F26 y, s;
#pragma unroll
          for (int w = 0; w < 5; ++w) y.a[w] = K[8 + 5 * b + w];
          const bool use = (m >> b) & 1u;
#pragma unroll
          for (int w = 0; w < 5; ++w) s.a[w] = use ? y.a[w] : (w == 0 ? 1u : 0u);
          h = mul26(h, s);
        }
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          // limbs < 2^26 + 2^9 after mul26: 16 of them fit in 32 bits, 64 do not
          if (b == 4) carry26(h);
#pragma unroll
          for (int w = 0; w < 5; ++w) h.a[w] += (uint32_t)__shfl_xor((int)h.a[w], 1 << b);
        }
        carry26(h);
        carry26(h);
        from26(h, p.h0, p.h1, p.h2, p.h3, p.h4);
        p.s0 = K[4]; p.s1 = K[5]; p.s2 = K[6]; p.s3 = K[7];
        poly_block(p, 0u, 0u, L, 0u);  // LE64(ad_len = 0) || LE64(len)
        poly_final(p, tag);
      }
      bool inpl = false;
      if (DECRYPT) {
        const uint4 want = load16<false>(rin + L, 16);
        const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) |
                              (want.w ^ tag[3]);
        ok = __builtin_amdgcn_readfirstlane((int)(diff == 0u)) != 0;
        inpl = rin == rout;
        if (lane == 0) a.status[di] = ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
      } else if (lane == 0) {
        store16<false>(rout + L, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
      }
      // ---- the windows out (decrypt: keystream first; a failed record: zeros
      // out of place, nothing in place), each followed by the next record's
#pragma unroll
      for (uint32_t k = 0; k < 2; ++k) {
        if (DECRYPT && ok) xor_win(k);
        wait_lds();  // the store instructions read other lanes' pieces
        wave_lds_fence();
        if (!DECRYPT || ok || !inpl) store_win(rout, k, DECRYPT && !ok);
        wait_lds();
        wave_lds_fence();
        if (has_next) load_win(a.in + nin, k);
      }
    }
    // the next super-tile's key pass overwrites kp; its windows are loaded
    // after it: every read of this one done
    wait_vmem();
    wait_lds();
    wave_lds_fence();
  }
}

}  // namespace noise_amd
