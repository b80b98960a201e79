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

template <bool DECRYPT>
__global__ __launch_bounds__(kOneBlock) void k_aead_one(const OneArgs a) {
#if defined(NOISE_HIP_EMU)
  uint4 *lds = reinterpret_cast<uint4 *>(emu::dyn_lds);  // tools/emu
#else
  extern __shared__ uint4 lds[];
#endif
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
        lds_dma16_v(src, (lds_void *)(lds + i0));
      }
    }
  }

  // 2. keystream: block b on thread b % 256; block 0 = one-time Poly key
  const uint32_t nlo = (uint32_t)a.nonce, nhi = (uint32_t)(a.nonce >> 32);
  const uint32_t nb = (L + 63u) >> 6;
  uint32_t ks[kOneMaxKsPerThread][16];
#pragma unroll
  for (int j = 0; j < kOneMaxKsPerThread; ++j) {
    const uint32_t b = t + (uint32_t)j * kOneBlock;
    if (b > nb) break;
    chacha20_block(a.key.w, b, nlo, nhi, ks[j]);
  }
  wait_vmem();  // this wave's DMA has landed ...
  __syncthreads();  // ... and every other wave's
#pragma unroll
  for (int j = 0; j < kOneMaxKsPerThread; ++j) {
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

  // 3. Poly1305 tree over P = na + nl + 1 blocks
  const uint32_t P = na + nl + 1u;
  const uint32_t NW = P > 256u ? 4u : 1u;  // waves taking part
  const uint32_t T = 64u * NW;
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
    for (uint32_t q = 0; q < c; ++q) {
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
    F26 R = pow26(to26(p.r0, p.r1, p.r2, p.r3, 0u), c);  // r^c
#pragma unroll
    for (int l = 0; l < 6; ++l) {
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

  // 4. LDS -> staging
  uint32_t *hdr = reinterpret_cast<uint32_t *>(base);
  if (!DECRYPT) {
    for (uint32_t i = t; i <= nl; i += kOneBlock) {  // ct pieces, then the tag
      const uint4 v = lds[i < nl ? na + i : s_tag];
      const u32x4 w = {v.x, v.y, v.z, v.w};
      *(g_u32x4 *)(base + lay.out + 16ull * i) = w;
    }
  } else {
    const bool ok = lds[s_ok].x == 0u;
    if (ok) {  // verified: apply the keystream held in registers, write plaintext
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
          *(g_u32x4 *)(base + lay.out + 16ull * p) = w;
        }
      }
    }
    if (t == 0) hdr[1] = ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC;
  }
  // 5. every store of the workgroup is visible system-wide before the done
  // word (stores -> system release -> drain -> barrier -> one flag store)
  __threadfence_system();
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the drain the compiler may drop
#endif
  __syncthreads();
  if (t == 0) __hip_atomic_store(hdr, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kMaxAttrDev = 64;

size_t one_lds_bytes(uint32_t ad_len, uint32_t len) {
  const uint32_t na = (ad_len + 15u) >> 4, nl = (len + 15u) >> 4;
  return 16ull * (na + nl + 4u + 8u);
}

hipError_t launch_aead_one(bool decrypt, const uint32_t key[8], uint64_t nonce,
                           uint8_t *d_base, uint32_t len, uint32_t ad_len, uint32_t seq,
                           hipStream_t stream) {
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
    attr_err[dev] = r;
  });
  if (attr_err[dev] != hipSuccess) return attr_err[dev];
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
