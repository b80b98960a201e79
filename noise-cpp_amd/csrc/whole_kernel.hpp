// whole_kernel.hpp -- records of 16 KiB < len <= 65535 B, one wave per
// record, lane-contiguous spans (records_kernels.hip, round 5).
//
// Noise decrypt checks a record's tag before any of its plaintext leaves
// (crypto_aead_read, monocypher.c:2912-2929).  The segment path spreads a
// long record's 1 KiB segments over the GPU, so its decrypt needs a Poly1305
// pass, a tag-check kernel and a keystream pass that reads the ciphertext a
// second time ~1 GB later.  Here one wave owns a whole record:
//   * lane j owns the contiguous span [j S, (j + 1) S) of the record, S =
//     256 B per 16 KiB of record (S = 512 B up to 32 KiB, 1 KiB up to 64 KiB),
//     so its Poly1305 sum is one Horner chain (BPL = S / 16 blocks) and its
//     keystream blocks are consecutive;
//   * the record passes through a 16 KiB LDS window in R = S / 256 rounds:
//     round k holds bytes [j S + 256 k, j S + 256 k + 256) of every span, one
//     LDS-DMA instruction per 16-byte piece column (lane l's piece q of the
//     round lands in slot 64 q + l: conflict-free ds_read_b128);
//   * decrypt: Poly1305 over the rounds, the tag (sum_j H_j r^(BPL (jl - j)),
//     jl the lane holding the last block), checked; then the rounds again
//     (the record's lines are ~64 KiB back: cache hits), keystream, and the
//     plaintext only if the tag verified (a failed record: zeros out of
//     place, nothing in place);
//   * encrypt: one pass, keystream and Poly1305 of the ciphertext per round,
//     then the tag.
// A super-tile is 8 records: lanes 0..7 compute their one-time keys and the
// powers r^(BPL 2^b) (b = 0..5) once, into LDS.
#pragma once
#include "tile_kernel.hpp"

namespace noise_amd {

constexpr int kWholeRPS = 8;  // records per super-tile

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
// lane's recombination weight r^(BPL m), m = 0..63, from r^(BPL 2^b)
__device__ __forceinline__ F26 whole_pow(const uint32_t *pw, uint32_t m) {
  F26 acc = {{1u, 0u, 0u, 0u, 0u}};
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    F26 y, s;
#pragma unroll
    for (int i = 0; i < 5; ++i) y.a[i] = pw[5 * b + i];
    const bool use = (m >> b) & 1u;
#pragma unroll
    for (int i = 0; i < 5; ++i) s.a[i] = use ? y.a[i] : (i == 0 ? 1u : 0u);
    acc = mul26(acc, s);
  }
  return acc;
}

template <bool DECRYPT>
__global__ __launch_bounds__(64) void k_whole(const TileArgs a) {
  __shared__ uint4 win[16 * 64];                 // one round: 16 pieces x 64 lanes
  __shared__ uint32_t kp[kWholeRPS][44];         // r[4], s[4], r^(BPL 2^b) [6][5], bad, r^nl [5]
  const uint32_t lane = threadIdx.x;
  const uint64_t base = a.cls_base[a.cls], n = a.counts[a.cls];

#pragma unroll 1
  for (uint64_t super0 = (uint64_t)blockIdx.x * kWholeRPS; super0 < n;
       super0 += (uint64_t)gridDim.x * kWholeRPS) {
    // ---- key pass: lane l < kWholeRPS -> record super0 + l -----------------
    uint32_t own_di = 0, own_len = 0, own_k[8];
    uint64_t own_n = 0, own_in = 0, own_out = 0;
    bool own_bad = true;
    {
      const uint64_t rec = super0 + lane;
      uint32_t ki = 0;
      if (lane < (uint32_t)kWholeRPS && rec < n) {
        own_di = a.idx[base + rec];
        const noise_gpu_record d = a.recs[own_di];
        ki = d.key_idx;
        own_n = d.nonce;
        own_in = d.in_off;
        own_out = d.out_off;
        own_len = d.len;
        own_bad = ki >= a.nkeys;
      }
      if (own_bad) ki = 0;
      const u32x4 *kp4 = reinterpret_cast<const u32x4 *>(a.keys + 32ull * ki);
      const u32x4 ka = kp4[0], kb = kp4[1];
      own_k[0] = ka.x; own_k[1] = ka.y; own_k[2] = ka.z; own_k[3] = ka.w;
      own_k[4] = kb.x; own_k[5] = kb.y; own_k[6] = kb.z; own_k[7] = kb.w;
      uint32_t otk[16];
      chacha20_block(own_k, 0u, (uint32_t)own_n, (uint32_t)(own_n >> 32), otk);
      if (lane < (uint32_t)kWholeRPS) {
        const uint32_t r0 = otk[0] & 0x0fffffffu, r1 = otk[1] & 0x0ffffffcu,
                       r2 = otk[2] & 0x0ffffffcu, r3 = otk[3] & 0x0ffffffcu;
        uint32_t *K = kp[lane];
        K[0] = r0; K[1] = r1; K[2] = r2; K[3] = r3;
        K[4] = otk[4]; K[5] = otk[5]; K[6] = otk[6]; K[7] = otk[7];
        // r^BPL, BPL = 16 S_k (S_k = span / 256 B = 1..4), and r^nl (nl = the
        // last lane's blocks, 1..BPL), by squaring: r^16, r^32, r^48, r^64
        // (lanes past the batch: len 0, nothing below is used)
        const uint32_t len1 = own_len ? own_len : 1u;
        const uint32_t sk = (len1 + 16383u) >> 14;  // 2..4 (16 KiB < len <= 65535)
        const uint32_t nblk = (len1 + 15u) >> 4, bpl = 16u * sk;
        const uint32_t nl = nblk - ((nblk - 1u) / bpl) * bpl;
        F26 x = to26(r0, r1, r2, r3, 0u), x16, x32, x64, rnl = {{1u, 0u, 0u, 0u, 0u}};
#pragma unroll
        for (int b = 0; b < 7; ++b) {
          rnl = mul26_if(rnl, x, ((nl >> b) & 1u) != 0u);
          if (b == 4) x16 = x;
          if (b == 5) x32 = x;
          if (b == 6) x64 = x;
          if (b < 6) x = mul26(x, x);
        }
        const F26 x48 = mul26(x32, x16);
        F26 y = sk <= 1u ? x16 : sk == 2u ? x32 : sk == 3u ? x48 : x64;
#pragma unroll
        for (int i = 0; i < 5; ++i) K[39 + i] = rnl.a[i];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
#pragma unroll
          for (int i = 0; i < 5; ++i) K[8 + 5 * b + i] = y.a[i];
          if (b < 5) y = mul26(y, y);
        }
        K[38] = own_bad ? 1u : 0u;
      }
    }
    wait_lds();
    wave_lds_fence();

#pragma unroll 1
    for (uint32_t i = 0; i < (uint32_t)kWholeRPS; ++i) {
      if (super0 + i >= n) break;
      // this record's fields, wave-uniform (SGPRs)
      const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)own_len, (int)i);
      const uint32_t di = (uint32_t)__builtin_amdgcn_readlane((int)own_di, (int)i);
      const uint64_t in_off = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_in >> 32), (int)i),
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_in, (int)i));
      const uint64_t out_off = join64((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_out >> 32), (int)i),
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_out, (int)i));
      const uint32_t n_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)own_n, (int)i);
      const uint32_t n_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(own_n >> 32), (int)i);
      const uint32_t *K = kp[i];
      if (K[38]) {  // bad key index: nothing written (status from the classifier's rule)
        if (DECRYPT && lane == 0) a.status[di] = NOISE_GPU_REC_BAD_KEY;
        continue;
      }
      uint32_t kt[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) kt[w] = (uint32_t)__builtin_amdgcn_readlane((int)own_k[w], (int)i);
      const uint32_t sk = (len + 16383u) >> 14;  // rounds (S = 256 sk bytes per lane)
      const uint32_t S = 256u * sk, BPL = 16u * sk;
      const uint32_t nblk = (len + 15u) >> 4;
      const uint32_t jl = (nblk - 1u) / BPL;  // the lane holding the last block
      const uint32_t lo = lane * S;           // my span's first byte
      // my span's bytes (0 past the record)
      const uint32_t myb = lo < len ? (len - lo < S ? len - lo : S) : 0u;
      const uint8_t *rin = a.in + in_off;
      uint8_t *rout = a.out + out_off;
      Poly1305 p;
      {
        uint32_t r[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) r[w] = K[w];
        p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
        p.r0 = r[0]; p.r1 = r[1]; p.r2 = r[2]; p.r3 = r[3];
        p.rr0 = (p.r0 >> 2) * 5u;
        p.rr1 = p.r1 + (p.r1 >> 2);
        p.rr2 = p.r2 + (p.r2 >> 2);
        p.rr3 = p.r3 + (p.r3 >> 2);
        p.r0lo = p.r0 & 3u;
      }
      // Round k of the window: span j's 256-byte chunk [j S + 256 k, +256)
      // sits in slots 16 j .. 16 j + 15, piece i at slot 16 j + (i ^ (j & 15))
      // (the tile kernel's swizzle: the owner's ds_read_b128 are conflict-
      // free).  Memory instruction q (DMA in, store out) moves the chunks of
      // spans 4q .. 4q + 3, 16 lanes each: lane l takes slot 64 q + l, i.e.
      // span jq = 4q + l / 16, piece iq = (l & 15) ^ (jq & 15) -- 256
      // contiguous bytes per 16 lanes.
      auto moff = [&](int q, uint32_t k) -> uint32_t {  // record byte of lane's piece in instruction q
        const uint32_t jq = 4u * (uint32_t)q + (lane >> 4);
        return jq * S + 256u * k + 16u * ((lane & 15u) ^ (jq & 15u));
      };
      auto load_round = [&](uint32_t k) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const uint32_t off = moff(q, k);
          // decrypt: a piece with any record byte is read whole (the last
          // one reads into the tag); encrypt: whole pieces by DMA, the
          // partial last one by bytes
          if (DECRYPT ? off < len : off + 16u <= len)
            lds_dma16_v<true>(rin + off, (lds_void *)NOISE_LDS3(win + 64 * q));
          else if (!DECRYPT && off < len)
            win[64u * q + lane] = load16<false>(rin + off, (int)(len - off));
        }
      };
      // the window -> HBM (out of place failed records: zeros)
      auto store_round = [&](uint32_t k, bool zero) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const uint32_t off = moff(q, k);
          if (off < len) {
            const uint4 v = zero ? make_uint4(0u, 0u, 0u, 0u) : win[64u * q + lane];
            if (off + 16u <= len) store16<true>(rout + off, v, 16);
            else store16<false>(rout + off, v, (int)(len - off));
          }
        }
      };
      const uint32_t sw = lane & 15u;
      // ---- decrypt: Poly1305 and the tag first ----------------------------
      bool ok = true;
      if (DECRYPT) {
#pragma unroll 1
        for (uint32_t k = 0; k < sk; ++k) {
          load_round(k);
          wait_vmem();
          wave_lds_fence();
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t off = 256u * k + 16u * i;  // in my span
            if (off < myb) {
              const uint32_t nb = myb - off;
              uint4 v = win[16u * lane + ((uint32_t)i ^ sw)];
              if (nb < 16u) v = mask_bytes(v, (int)nb);
              poly_block(p, v.x, v.y, v.z, v.w);
            }
          }
          wait_lds();
          wave_lds_fence();
        }
      }
      // the keystream over round k's pieces of my span, into the window;
      // encrypt: Poly1305 of the ciphertext as it goes
      const ChaPre pre = chacha_pre(kt, n_lo, n_hi);
      auto xor_round = [&](uint32_t k) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {  // the round's four 64-byte keystream blocks
          const uint32_t off0 = 256u * k + 64u * c;
          uint32_t ks[16];
          chacha20_block_pre(kt, 1u + ((lo + off0) >> 6), pre, n_lo, n_hi, ks);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const uint32_t i = 4u * (uint32_t)c + (uint32_t)qq, off = off0 + 16u * (uint32_t)qq;
            if (off < myb) {
              const uint32_t nb = myb - off;
              const uint32_t slot = 16u * lane + (i ^ sw);
              const uint4 v = win[slot];
              uint4 o = make_uint4(v.x ^ ks[4 * qq + 0], v.y ^ ks[4 * qq + 1], v.z ^ ks[4 * qq + 2],
                                   v.w ^ ks[4 * qq + 3]);
              if (nb < 16u) o = mask_bytes(o, (int)nb);
              if (!DECRYPT) poly_block(p, o.x, o.y, o.z, o.w);
              win[slot] = o;
            }
          }
        }
      };
      if (!DECRYPT) {
#pragma unroll 1
        for (uint32_t k = 0; k < sk; ++k) {
          load_round(k);
          wait_vmem();
          wave_lds_fence();
          xor_round(k);
          wait_lds();  // the store instructions read other lanes' pieces
          wave_lds_fence();
          store_round(k, false);
          wait_lds();
          wave_lds_fence();
        }
      }
      // ---- the tag: sum_j H_j r^(weight) + the length block ----------------
      {
        // lane j < jl: its span's blocks end BPL (jl - 1 - j) + nl before the
        // record's last (nl: the last lane's blocks), lane jl: at it
        F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
        h = mul26(h, whole_pow(K + 8, lane < jl ? jl - 1u - lane : 0u));
        h = mul26_if(h, f26_load(K + 39), lane < jl);
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
        poly_block(p, 0u, 0u, len, 0u);  // LE64(ad_len = 0) || LE64(len)
        uint32_t tag[4];
        poly_final(p, tag);
        if (DECRYPT) {
          const uint4 want = load16<false>(rin + len, 16);
          const uint32_t diff = (want.x ^ tag[0]) | (want.y ^ tag[1]) | (want.z ^ tag[2]) |
                                (want.w ^ tag[3]);
          ok = __builtin_amdgcn_readfirstlane((int)(diff == 0u)) != 0;
          if (lane == 0) a.status[di] = ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
        } else if (lane == 0) {
          store16<false>(rout + len, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
        }
      }
      // ---- decrypt: the rounds again, keystream, verified plaintext --------
      if (DECRYPT) {
        const bool inpl = rin == rout;
        if (!ok && inpl) continue;  // a failed record decrypted in place: untouched
#pragma unroll 1
        for (uint32_t k = 0; k < sk; ++k) {
          if (ok) {
            load_round(k);
            wait_vmem();
            wave_lds_fence();
            xor_round(k);
            wait_lds();
            wave_lds_fence();
          }
          store_round(k, !ok);
          wait_lds();
          wave_lds_fence();
        }
      }
    }
    // the next super-tile's key pass overwrites kp: every lane's reads done
    wait_lds();
    wave_lds_fence();
  }
}

}  // namespace noise_amd
