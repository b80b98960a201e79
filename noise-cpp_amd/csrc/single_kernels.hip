// single_kernels.hip -- the latency path: ONE record per workgroup, read from
// and written to host-mapped pinned staging (noise_gpu_encrypt_host /
// _decrypt_host / _rekey_host, i.e. CipherState::encrypt_with_ad /
// decrypt_with_ad / rekey and every handshake payload).
//
// The reference does one record per call on the CPU (noise.cpp:393-427 ->
// monocypher.c:2899-2929).  Here one call = one kernel launch and no copy
// engine: the workgroup pulls the staged AD and record straight over PCIe
// into LDS (LDS-DMA, all pieces in flight at once, landing while the
// keystream is computed), spreads the work over 256 lanes
// and pushes the result back the same way, then raises a completion word in
// the staging header that the host polls (no hipMemcpyAsync pair, no stream
// synchronisation on the fast path).
//
//   * ChaCha20: keystream block b on thread b mod 256 (block 0 = the
//     Poly1305 key, monocypher.c:2903); a 1 KiB record is one block per lane.
//   * Poly1305 over AD || pad || ct || pad || LE64(A) || LE64(L)
//     (monocypher.c:2858-2873) as a tree: the P blocks are right-aligned in
//     T = 64 (or 256) chunks of c = ceil(P/T) blocks; each lane Horner-
//     evaluates its chunk with the clamped r (radix 2^32), then the chunks
//     combine pairwise, left * r^(c 2^l) + right, over log2 T levels
//     (shuffles within a wave, LDS across waves).
//   * Decrypt verifies the tag before any plaintext leaves the workgroup
//     (crypto_aead_read, monocypher.c:2912-2929): the keystream blocks stay
//     in registers until the verdict; a failed record writes nothing.
//
// Staging layout (shared with the host, one_layout() in launchers.hpp):
//   [0,64)   header: u32 done word, u32 status
//   ad       A bytes, zero padded to 16
//   in       L bytes (plaintext / ciphertext), zero padded to 16
//   tag      16 bytes (decrypt: the received tag)
//   out      ciphertext padded to 16 + tag (encrypt) / plaintext (decrypt)
#include <mutex>

#include "chachapoly_device.hpp"
#include "launchers.hpp"

namespace noise_amd {

constexpr int kOneBlock = 256;
// keystream blocks 0..ceil(65535 / 64) = 1025 blocks over 256 threads
constexpr int kOneMaxKsPerThread = ((65535 + 63) / 64 + 1 + kOneBlock - 1) / kOneBlock;
static_assert(kOneMaxKsPerThread == 5, "blocks per thread of a 65535-byte record");

struct OneArgs {
  KeyArg key;
  uint64_t nonce;
  uint8_t *base;  // device-visible address of the staging image
  uint32_t len, ad_len;
  uint32_t seq;   // written to the done word last
};

// 16 bytes to the host-mapped staging image with ONE system-scope,
// write-through store (buffer_store_dwordx4 ... sc0 sc1), emitted by the
// compiler so its VGPR hazards and vmcnt bookkeeping stay the compiler's.
// (An inline-asm global_store_dwordx4 sc0 sc1 lost data: the compiler reused
// its data VGPRs before the store had read them.  Two 8-byte atomic stores
// instead cost ~8 us per 64 KiB record over PCIe.)  Buffer-resource word 3:
// 0x00020000, the gfx9-family raw-buffer format (as in CK).
__device__ __forceinline__ void st_sys16(uint8_t *base, uint64_t off, u32x4 w) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t img = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(w, img, (int)off, 0, 1 | 16);  // aux: sc0 (glc) | sc1 (scc)
#else
  *(g_u32x4 *)(base + off) = w;
#endif
}

// x * y by binary exponentiation: x^e (e >= 1)
__device__ __forceinline__ F26 pow26(F26 x, uint32_t e) {
  F26 r = x;
  const int top = 31 - __builtin_clz(e);
  for (int b = top - 1; b >= 0; --b) {
    r = mul26(r, r);
    if ((e >> b) & 1u) r = mul26(r, x);
  }
  return r;
}

__device__ __forceinline__ F26 add26(const F26 &a, const F26 &b) {
  F26 r;
#pragma unroll
  for (int i = 0; i < 5; ++i) r.a[i] = a.a[i] + b.a[i];
  return r;
}

// One record, the whole workgroup (k_aead_one: one launch per record;
// k_aead_resident: a resident workgroup serving a doorbell ring).
// tools/ubench/one_timing.hip builds this file with NOISE_ONE_TIMING: thread
// 0 stamps s_memrealtime at the phase boundaries into the done line
#ifdef NOISE_ONE_TIMING
#define NOISE_ONE_STAMP(i)                                                       \
  if (threadIdx.x == 0)                                                          \
    reinterpret_cast<uint64_t *>(a.base)[2 + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define NOISE_ONE_STAMP(i) ((void)0)
#endif

template <bool DECRYPT>
__device__ __forceinline__ void one_body(const OneArgs &a, uint4 *lds) {
  NOISE_ONE_STAMP(0);
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  const uint32_t L = a.len, A = a.ad_len;
  const uint32_t na = (A + 15u) >> 4, nl = (L + 15u) >> 4;
  const OneLayout lay = one_layout(A, L);
  uint8_t *base = a.base;
  // LDS: [0,na) AD pieces, [na,na+nl) record pieces, na+nl the tag, then
  // r, s, the verdict and 4 x 2 slots of per-wave Poly1305 sums
  const uint32_t s_tag = na + nl, s_r = s_tag + 1, s_s = s_r + 1, s_ok = s_s + 1, s_w = s_ok + 1;

  // 1. staging -> LDS by LDS-DMA: AD, record and (decrypt) tag pieces land
  // at lds[0..npc) without passing through registers, so nothing waits for
  // the PCIe round trip until the keystream blocks below are computed
  {
    const uint32_t npc = na + nl + (DECRYPT ? 1u : 0u);
    // wave-uniform base (readfirstlane: M0 takes an SGPR)
    for (uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(wave * 64u)); i0 < npc;
         i0 += kOneBlock) {
      const uint32_t i = i0 + lane;
      if (i < npc) {
        const uint8_t *src = base + (i < na ? lay.ad + 16ull * i : lay.in + 16ull * (i - na));
        lds_dma16_v_sys(src, (lds_void *)(lds + i0));  // the host rewrote it: bypass caches
      }
    }
  }

  // 2. keystream; block 0 = one-time Poly key.  Records of <= 63 data
  // blocks (4032 B): block b on the quad of threads 4b..4b+3 (chacha20_quad,
  // a third of one lane's latency; thread 4b + q holds column q).  Longer
  // ones: block b on thread b % 256.
  const uint32_t nlo = (uint32_t)a.nonce, nhi = (uint32_t)(a.nonce >> 32);
  const uint32_t nb = (L + 63u) >> 6;
  const bool quad = nb < 64u;  // workgroup-uniform
  uint32_t ks[kOneMaxKsPerThread][16];
  uint32_t kq[4] = {0u, 0u, 0u, 0u};
  uint32_t *lds32 = reinterpret_cast<uint32_t *>(lds);
  if (quad) {
    // every quad runs (blocks past nb unused): no divergence around the DPP
    chacha20_quad(a.key.w, t & 3u, t >> 2, nlo, nhi, kq);
  } else {
#pragma unroll
    for (int j = 0; j < kOneMaxKsPerThread; ++j) {
      const uint32_t b = t + (uint32_t)j * kOneBlock;
      if (b > nb) break;
      chacha20_block(a.key.w, b, nlo, nhi, ks[j]);
    }
  }
  NOISE_ONE_STAMP(1);
  wait_vmem();  // this wave's DMA has landed ...
  __syncthreads();  // ... and every other wave's
  // quad: thread (b, q) holds keystream words 4r + q (r = 0..3) of block b,
  // i.e. word q of pieces 4(b-1) + r; XOR word-wise in LDS
  auto quad_xor = [&](bool to_ct) {
    const uint32_t b = t >> 2, q = t & 3u;
    if (b == 0 || b > nb) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t p = 4u * (b - 1u) + (uint32_t)r;
      if (p >= nl) break;
      const int nbytes = (int)(L - 16u * p - 4u * q);  // bytes of this word in the record
      if (nbytes <= 0) {
        if (to_ct) lds32[4u * (na + p) + q] = 0u;  // padding of the last piece: zero
        continue;
      }
      const uint32_t m = nbytes >= 4 ? 0xffffffffu : (1u << (8 * nbytes)) - 1u;
      lds32[4u * (na + p) + q] = (lds32[4u * (na + p) + q] ^ kq[r]) & m;
    }
  };
  if (quad) {
    if (t < 4u) {  // block 0: r (clamped) = row 0, s = row 1
      const uint32_t cm = t == 0 ? 0x0fffffffu : 0x0ffffffcu;
      lds32[4u * s_r + t] = kq[0] & cm;
      lds32[4u * s_s + t] = kq[1];
    }
    if (!DECRYPT) quad_xor(true);
  }
#pragma unroll
  for (int j = 0; j < kOneMaxKsPerThread; ++j) {
    if (quad) break;
    const uint32_t b = t + (uint32_t)j * kOneBlock;
    if (b > nb) break;
    if (b == 0) {
      lds[s_r] = make_uint4(ks[j][0] & 0x0fffffffu, ks[j][1] & 0x0ffffffcu,
                            ks[j][2] & 0x0ffffffcu, ks[j][3] & 0x0ffffffcu);
      lds[s_s] = make_uint4(ks[j][4], ks[j][5], ks[j][6], ks[j][7]);
    } else if (!DECRYPT) {  // plaintext -> ciphertext in LDS (bytes past L stay 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t p = 4u * (b - 1u) + (uint32_t)q;
        if (p >= nl) break;
        const int nbytes = (int)(L - 16u * p) >= 16 ? 16 : (int)(L - 16u * p);
        const uint4 v = lds[na + p];
        lds[na + p] = mask_bytes(make_uint4(v.x ^ ks[j][4 * q], v.y ^ ks[j][4 * q + 1],
                                            v.z ^ ks[j][4 * q + 2], v.w ^ ks[j][4 * q + 3]),
                                 nbytes);
      }
    }
  }
  __syncthreads();

  NOISE_ONE_STAMP(2);
  // 3. Poly1305 tree over P = na + nl + 1 blocks
  const uint32_t P = na + nl + 1u;
  const uint32_t NW = P > 256u ? 4u : 1u;  // waves taking part
  // Tree width T = 2^LT lanes: the latency is ~c Horner steps plus LT tree
  // levels (a general product, its carry and the power squaring: ~2.2 Horner
  // steps each), so short records use a narrow tree -- one lane for <= ~8
  // blocks -- instead of 64 lanes and six levels.  Above 256 blocks: four
  // full waves.
  uint32_t LT = 6;
  if (NW == 1) {
    uint32_t best = ~0u;
#pragma unroll
    for (uint32_t l = 0; l <= 6; ++l) {
      const uint32_t cost = ((P + (1u << l) - 1u) >> l) * 10u + l * 22u;
      if (cost < best) {
        best = cost;
        LT = l;
      }
    }
  }
  const uint32_t T = NW == 1 ? (1u << LT) : 64u * NW;
  const uint32_t c = (P + T - 1u) / T;    // blocks per chunk
  const uint32_t pad = T * c - P;         // leading empty positions
  if (wave < NW) {
    const uint4 rv = lds[s_r];
    Poly1305 p;
    p.r0 = rv.x; p.r1 = rv.y; p.r2 = rv.z; p.r3 = rv.w;
    p.rr0 = (p.r0 >> 2) * 5u;
    p.rr1 = p.r1 + (p.r1 >> 2);
    p.rr2 = p.r2 + (p.r2 >> 2);
    p.rr3 = p.r3 + (p.r3 >> 2);
    p.r0lo = p.r0 & 3u;
    p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
    const uint32_t j = wave * 64u + lane;
    for (uint32_t q = 0; q < (j < T ? c : 0u); ++q) {
      const uint32_t pos = j * c + q;
      if (pos < pad) continue;
      const uint32_t k = pos - pad;  // real block index
      if (k + 1u < P) {
        const uint4 m = lds[k];      // AD and record pieces are contiguous
        poly_block(p, m.x, m.y, m.z, m.w);
      } else {
        poly_block(p, A, 0u, L, 0u);  // LE64(ad_len) || LE64(len)
      }
    }
    F26 h = to26(p.h0, p.h1, p.h2, p.h3, p.h4);
    F26 R = to26(p.r0, p.r1, p.r2, p.r3, 0u);
    if (LT) R = pow26(R, c);  // r^c (unused by a one-lane Horner)
    for (uint32_t l = 0; l < LT; ++l) {  // wave-uniform trip count
      F26 right;
#pragma unroll
      for (int i = 0; i < 5; ++i) right.a[i] = (uint32_t)__shfl_down((int)h.a[i], 1 << l);
      h = add26(mul26(h, R), right);  // meaningful on lanes = 0 mod 2^(l+1)
      carry26(h);
      R = mul26(R, R);
    }
    if (NW > 1) {  // R = r^(64 c): combine the wave sums in order on wave 0
      if (lane == 0) {
        lds[s_w + 2 * wave] = make_uint4(h.a[0], h.a[1], h.a[2], h.a[3]);
        lds[s_w + 2 * wave + 1] = make_uint4(h.a[4], 0u, 0u, 0u);
      }
    }
    if (NW == 1 && lane == 0) {
      carry26(h);
      carry26(h);
      from26(h, p.h0, p.h1, p.h2, p.h3, p.h4);
      const uint4 sv = lds[s_s];
      p.s0 = sv.x; p.s1 = sv.y; p.s2 = sv.z; p.s3 = sv.w;
      uint32_t tag[4];
      poly_final(p, tag);
      if (!DECRYPT) {
        lds[s_tag] = make_uint4(tag[0], tag[1], tag[2], tag[3]);
      } else {
        const uint4 w = lds[s_tag];
        const uint32_t diff = (w.x ^ tag[0]) | (w.y ^ tag[1]) | (w.z ^ tag[2]) | (w.w ^ tag[3]);
        lds[s_ok] = make_uint4(diff, 0u, 0u, 0u);
      }
    }
    if (NW > 1) {
      __syncthreads();  // only reached when NW = 4: every wave takes part
      if (t == 0) {
        F26 H;
        const uint4 w0 = lds[s_w], w1 = lds[s_w + 1];
        H.a[0] = w0.x; H.a[1] = w0.y; H.a[2] = w0.z; H.a[3] = w0.w; H.a[4] = w1.x;
        for (uint32_t w = 1; w < NW; ++w) {
          const uint4 v0 = lds[s_w + 2 * w], v1 = lds[s_w + 2 * w + 1];
          F26 X;
          X.a[0] = v0.x; X.a[1] = v0.y; X.a[2] = v0.z; X.a[3] = v0.w; X.a[4] = v1.x;
          H = add26(mul26(H, R), X);
          carry26(H);
        }
        carry26(H);
        carry26(H);
        from26(H, p.h0, p.h1, p.h2, p.h3, p.h4);
        const uint4 sv = lds[s_s];
        p.s0 = sv.x; p.s1 = sv.y; p.s2 = sv.z; p.s3 = sv.w;
        uint32_t tag[4];
        poly_final(p, tag);
        if (!DECRYPT) {
          lds[s_tag] = make_uint4(tag[0], tag[1], tag[2], tag[3]);
        } else {
          const uint4 w = lds[s_tag];
          const uint32_t diff = (w.x ^ tag[0]) | (w.y ^ tag[1]) | (w.z ^ tag[2]) | (w.w ^ tag[3]);
          lds[s_ok] = make_uint4(diff, 0u, 0u, 0u);
        }
      }
    }
  }
  __syncthreads();

  NOISE_ONE_STAMP(3);
  // 4. LDS -> staging
  uint32_t *hdr = reinterpret_cast<uint32_t *>(base);
  if (!DECRYPT) {
    for (uint32_t i = t; i <= nl; i += kOneBlock) {  // ct pieces, then the tag
      const uint4 v = lds[i < nl ? na + i : s_tag];
      const u32x4 w = {v.x, v.y, v.z, v.w};
      st_sys16(base, lay.out + 16ull * i, w);
    }
  } else {
    const bool ok = lds[s_ok].x == 0u;
    if (ok && quad) {  // verified: keystream (registers) into LDS, then pieces out
      quad_xor(false);
      __syncthreads();
      for (uint32_t i = t; i < nl; i += kOneBlock) {
        const uint4 v = lds[na + i];
        const u32x4 w = {v.x, v.y, v.z, v.w};
        st_sys16(base, lay.out + 16ull * i, w);
      }
    }
    if (ok && !quad) {  // verified: apply the keystream held in registers, write plaintext
#pragma unroll
      for (int j = 0; j < kOneMaxKsPerThread; ++j) {
        const uint32_t b = t + (uint32_t)j * kOneBlock;
        if (b > nb) break;
        if (b == 0) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t p = 4u * (b - 1u) + (uint32_t)q;
          if (p >= nl) break;
          const int nbytes = (int)(L - 16u * p) >= 16 ? 16 : (int)(L - 16u * p);
          const uint4 v = lds[na + p];
          const uint4 o = mask_bytes(make_uint4(v.x ^ ks[j][4 * q], v.y ^ ks[j][4 * q + 1],
                                                v.z ^ ks[j][4 * q + 2], v.w ^ ks[j][4 * q + 3]),
                                     nbytes);
          const u32x4 w = {o.x, o.y, o.z, o.w};
          st_sys16(base, lay.out + 16ull * p, w);
        }
      }
    }
    if (t == 0)
      __hip_atomic_store(hdr + 1, ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  NOISE_ONE_STAMP(4);
  // 5. every store of the workgroup is visible system-wide before the done
  // word (stores -> system release -> drain -> barrier -> one flag store)
  // Every output store above is a system-scope write-through store (sc0
  // sc1) to the host-mapped image, so draining them (vmcnt(0)) is the whole
  // release: no L2 write-back (buffer_wbl2, ~1.4 us) is needed before the
  // done word (MI355X_MICROARCH.md: sc1 stores drained before the flag).
#ifdef NOISE_ONE_SYSFENCE  // A/B (tools/ubench/one_timing): the full system release
  __threadfence_system();
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  __syncthreads();
  NOISE_ONE_STAMP(5);
  if (t == 0) __hip_atomic_store(hdr, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool DECRYPT>
__global__ __launch_bounds__(kOneBlock) void k_aead_one(const OneArgs a) {
#if defined(NOISE_HIP_EMU)
  uint4 *lds = reinterpret_cast<uint4 *>(emu::dyn_lds);  // tools/emu
#else
  extern __shared__ uint4 lds[];
#endif
  one_body<DECRYPT>(a, lds);
}

// ---- resident latency kernel (opt-in: noise_gpu_set_resident) -------------
// One workgroup stays on the GPU and serves requests from the host-mapped
// staging image instead of one launch per record: the host writes the AD /
// record as above plus the request line (key, nonce, lengths, direction;
// OneRing in launchers.hpp), then bumps the doorbell; lane 0 polls the
// doorbell over PCIe (system-scope loads, s_sleep between polls), the
// workgroup runs one_body and raises the done word exactly like k_aead_one.
// Every wave leaves the loop together (the decision goes through LDS) when
//   * the stop word is set (noise_gpu_set_resident(0), context teardown,
//     thread exit), or
//   * no request has arrived for `idle_ticks` of the 100 MHz s_memrealtime
//     clock -- so the grid always drains on its own, even if the host never
//     stops it; the host relaunches it on the next request.
// `last` is the doorbell value already served when this instance started: a
// request rung while an idle instance was exiting is picked up by the next.
__global__ __launch_bounds__(kOneBlock) void k_aead_resident(uint8_t *base, uint32_t last,
                                                             uint64_t idle_ticks) {
#if defined(NOISE_HIP_EMU)
  uint4 *lds = reinterpret_cast<uint4 *>(emu::dyn_lds);  // tools/emu
#else
  extern __shared__ uint4 lds[];
#endif
  __shared__ uint64_t cmd[2];
  OneRing *ring = reinterpret_cast<OneRing *>(base + kOneRingOff);
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x == 0) {
      uint64_t db = 0, ex = 0;
      for (;;) {
        db = __hip_atomic_load(&ring->doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)db != last) break;
        if (__hip_atomic_load(&ring->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
            __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) {
          ex = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      cmd[0] = db;
      cmd[1] = ex;
    }
    __syncthreads();
    const uint64_t db = cmd[0], ex = cmd[1];
    __syncthreads();  // cmd is rewritten only after every thread has read it
    if (ex) break;
    // the rest of the request line (nonce, key) was written before the
    // doorbell: three 16-byte system-scope loads, all in flight together
    u32x4 q[3];
    {
      const u32x4 *rq = reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(ring) + 16);
#if defined(__HIP_DEVICE_COMPILE__)
      asm volatile("global_load_dwordx4 %0, %3, off sc0 sc1\n\t"
                   "global_load_dwordx4 %1, %3, off offset:16 sc0 sc1\n\t"
                   "global_load_dwordx4 %2, %3, off offset:32 sc0 sc1\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]) : "v"(rq) : "memory");
#else
      for (int i = 0; i < 3; ++i) q[i] = rq[i];
#endif
    }
    OneArgs a;
    a.nonce = ((uint64_t)q[0].y << 32) | q[0].x;
    a.key.w[0] = q[1].x; a.key.w[1] = q[1].y; a.key.w[2] = q[1].z; a.key.w[3] = q[1].w;
    a.key.w[4] = q[2].x; a.key.w[5] = q[2].y; a.key.w[6] = q[2].z; a.key.w[7] = q[2].w;
    a.base = base;
    a.len = (uint32_t)(db >> 32) & 0xffffu;
    a.ad_len = (uint32_t)(db >> 48) & 0x3fffu;
    const uint32_t dec = (uint32_t)(db >> 62) & 1u;
    a.seq = (uint32_t)db;
    if (a.ad_len > kOneMaxAd) a.ad_len = 0;  // the host never rings such a request
    if (dec) one_body<true>(a, lds);
    else one_body<false>(a, lds);
#pragma unroll
    for (int i = 0; i < 8; ++i) a.key.w[i] = 0u;
    last = a.seq;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  // gone: the host's unload hook waits for this word (done line, offset 8)
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(reinterpret_cast<uint32_t *>(base + 8), 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

constexpr int kMaxAttrDev = 64;

size_t one_lds_bytes(uint32_t ad_len, uint32_t len) {
  const uint32_t na = (ad_len + 15u) >> 4, nl = (len + 15u) >> 4;
  return 16ull * (na + nl + 4u + 8u);
}

static hipError_t one_attr() {
  // > 64 KiB of dynamic LDS needs the opt-in, which is per device: set once
  // per device, race-free across threads
  static std::once_flag attr_once[kMaxAttrDev];
  static hipError_t attr_err[kMaxAttrDev];
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxAttrDev) return hipErrorInvalidDevice;
  std::call_once(attr_once[dev], [dev] {
    const int max_lds = (int)one_lds_bytes(kOneMaxAd, 65535u);
    hipError_t r = hipFuncSetAttribute((const void *)k_aead_one<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, max_lds);
    if (r == hipSuccess)
      r = hipFuncSetAttribute((const void *)k_aead_one<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds);
    if (r == hipSuccess)
      r = hipFuncSetAttribute((const void *)k_aead_resident,
                              hipFuncAttributeMaxDynamicSharedMemorySize, max_lds);
    attr_err[dev] = r;
  });
  return attr_err[dev];
}

hipError_t launch_aead_resident(uint8_t *d_base, uint32_t last, uint32_t idle_us,
                                hipStream_t stream) {
  const hipError_t e = one_attr();
  if (e != hipSuccess) return e;
  const size_t lds = one_lds_bytes(kOneMaxAd, 65535u);
  hipLaunchKernelGGL(k_aead_resident, dim3(1), dim3(kOneBlock), lds, stream, d_base, last,
                     (uint64_t)idle_us * 100ull);  // s_memrealtime: 100 MHz
  return hipGetLastError();
}

hipError_t launch_aead_one(bool decrypt, const uint32_t key[8], uint64_t nonce,
                           uint8_t *d_base, uint32_t len, uint32_t ad_len, uint32_t seq,
                           hipStream_t stream) {
  const hipError_t e0 = one_attr();
  if (e0 != hipSuccess) return e0;
  OneArgs a;
  for (int i = 0; i < 8; ++i) a.key.w[i] = key[i];
  a.nonce = nonce;
  a.base = d_base;
  a.len = len;
  a.ad_len = ad_len;
  a.seq = seq;
  const size_t lds = one_lds_bytes(ad_len, len);
  if (decrypt)
    hipLaunchKernelGGL((k_aead_one<true>), dim3(1), dim3(kOneBlock), lds, stream, a);
  else
    hipLaunchKernelGGL((k_aead_one<false>), dim3(1), dim3(kOneBlock), lds, stream, a);
  for (int i = 0; i < 8; ++i) a.key.w[i] = 0u;
  return hipGetLastError();
}

}  // namespace noise_amd
