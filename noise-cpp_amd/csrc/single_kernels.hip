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
  uint8_t *base;        // device-visible address of the staging image (done line, output)
  uint8_t *in_base;     // where AD / record / tag are staged: base, or the resident
                        // kernel's request image in device memory
  uint32_t len, ad_len;
  uint32_t seq;         // written to the done word last
  uint32_t wipe_in;     // zero the staged input (request image) before the done word
  uint32_t staged;      // the input is already in (or on its way into) LDS: the
                        // resident kernel's polling wave unpacked or issued it
  uint8_t *req;         // resident: the request image (header / inline chunks)
  uint32_t n_inl;       // resident: inline chunks of this request (zeroed after use)
  uint32_t dec;         // RT bodies: the direction (the resident kernel's one copy)
};

// The staged input pieces [0, npc) -> LDS[0, npc) by LDS-DMA (AD pieces, then
// record pieces and, for decrypt, the tag: contiguous in the image), by the
// calling threads in rounds of `nthr` (64: one wave; 256: the workgroup).
// System-scope, cache-bypassing loads: the host rewrote the image.
__device__ __forceinline__ void one_stage_in(const uint8_t *in_base, const OneLayout &lay,
                                             uint32_t npc, uint4 *lds, uint32_t t, uint32_t nthr) {
  const uint32_t lane = t & 63u;
  // wave-uniform base (readfirstlane: M0 takes an SGPR)
  for (uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t & ~63u)); i0 < npc; i0 += nthr) {
    const uint32_t i = i0 + lane;
    if (i < npc) lds_dma16_v_sys(in_base + lay.ad + 16ull * i, (lds_void *)(lds + i0));
  }
}

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

// The resident kernel's request image after use: the header chunks keep
// only their seq word, the inline chunks are zeroed (threads u of nthr)
__device__ __forceinline__ void req_wipe(const OneArgs &a, uint32_t u, uint32_t nthr) {
  if (u < 4) {
    const u32x4 w = {a.seq, 0u, 0u, 0u};
    st_sys16(a.req, 16ull * u, w);
  }
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (uint32_t k = u; k < a.n_inl; k += nthr) st_sys16(a.req, 16ull * (4u + k), z);
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

// Step 5 of every single-record body: the resident kernel's request image
// is zeroed (the key words of the request line -- its sequence words stay --
// and the npc staged input pieces), then every store of the workgroup is
// visible system-wide before the done word (stores -> drain -> barrier -> one
// flag store).  Every store above is a system-scope write-through store (sc0
// sc1), so draining them (vmcnt(0)) is the whole release: no L2 write-back
// (buffer_wbl2, ~1.4 us) is needed before the done word (MI355X_MICROARCH.md:
// sc1 stores drained before the flag).  The zeroing must land before the
// done word too: the host writes the next request only after it.
__device__ __forceinline__ void one_finish(const OneArgs &a, const OneLayout &lay, uint32_t npc) {
  const uint32_t t = threadIdx.x;
  if (a.wipe_in) {
    const u32x4 z = {0u, 0u, 0u, 0u};
    if (!a.n_inl)
      for (uint32_t i = t; i < npc; i += kOneBlock) st_sys16(a.in_base, lay.ad + 16ull * i, z);
    req_wipe(a, t, kOneBlock);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(reinterpret_cast<uint32_t *>(a.base), a.seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// One record, the whole workgroup (k_aead_one: one launch per record;
// k_aead_resident: a resident workgroup serving a doorbell ring).

// RT (the resident kernel): ONE copy for both directions (a.dec at run time)
// and only the quad keystream path -- the kernel serves records of <= 63
// keystream blocks (bigger ones take the launch path) and must stay small:
// its poll loop, bodies and speculation share one instruction cache.
template <bool DECRYPT_T, bool RT = false>
__device__ __forceinline__ void one_body(const OneArgs &a, uint4 *lds) {
  const bool DECRYPT = RT ? a.dec != 0u : DECRYPT_T;
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
  if (!a.staged) one_stage_in(a.in_base, lay, na + nl + (DECRYPT ? 1u : 0u), lds, t, kOneBlock);

  // 2. keystream; block 0 = one-time Poly key.  Records of <= 63 data
  // blocks (4032 B): block b on the quad of threads 4b..4b+3 (chacha20_quad,
  // a third of one lane's latency; thread 4b + q holds column q).  Longer
  // ones: block b on thread b % 256.
  const uint32_t nlo = (uint32_t)a.nonce, nhi = (uint32_t)(a.nonce >> 32);
  const uint32_t nb = (L + 63u) >> 6;
  const bool quad = RT || nb < 64u;  // workgroup-uniform
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
  one_finish(a, lay, na + nl + (DECRYPT ? 1u : 0u));
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
// One workgroup stays on the GPU and serves the thread's single records
// instead of one launch per record.
//
//   * Requests arrive in a REQUEST IMAGE in device memory that the host
//     writes through the PCIe BAR (write-combined stores; launchers.hpp
//     OneReq): the AD / record / tag at one_layout() offsets, then the
//     request line -- four 16-byte chunks {seq, three payload words}: lengths
//     and direction, the nonce, the key.  Lanes 0..3 of wave 0 poll the four
//     chunks (system-scope loads, local memory: ~1 us per poll instead of a
//     PCIe round trip) and take a request when all four carry a new seq; the
//     host stores the chunks after an sfence that follows the data, and PCIe
//     keeps posted writes in order, so everything else has landed by then.
//   * Output, status and the done word go to the host-mapped image (write-
//     through stores) exactly as in the launch path; the request image is
//     zeroed (but for the chunks' seq words) before the done word.
//   * SPECULATION.  Noise sends consecutive nonces under one key, so after
//     answering (key, n) the workgroup precomputes for (key, n + 1) while the
//     host turns round: ChaCha blocks 0..63 of that nonce (one block per quad
//     of lanes, chacha20_quad) and the Poly1305 powers r, r^2 .. r^256 (nine
//     levels of products).  A request that matches a slot (key and nonce;
//     two slots, least recently used replaced, for a session's send and
//     receive keys) of <= 63 keystream blocks and <= 256 Poly1305 blocks
//     then costs only its data load, one XOR and ONE product per 16-byte
//     block -- sum_t m_t r^(P-t) in parallel over the 256 lanes, reduced by
//     shuffles -- instead of the block-0 -> r -> Horner-tree chain
//     (one_body_fast).  Anything else runs one_body.
//   * Every wave leaves the loop together (the decision goes through LDS)
//     when the stop word in the host image is set (polled every 32 polls), or
//     no request has arrived for `idle_ticks` of the 100 MHz s_memrealtime
//     clock -- so the grid always drains on its own.  On the way out the
//     speculation slots (future keystream, key copies) are zeroed in LDS.
// `last` is the seq already served when this instance started: a request
// rung while an idle instance was exiting is picked up by the next one.
constexpr uint32_t kSpecBlocks = 64;   // keystream blocks 1..63 of the next nonce
constexpr uint32_t kSpecPowers = 256;  // r^1 .. r^256
constexpr uint32_t kSpecSlots = 2;     // speculated (key, nonce)s: a session's two directions
constexpr uint32_t kSpecBufs = 3;      // tables: one per slot + the one being filled
constexpr uint32_t kFastMaxBlocks = 192;  // Poly1305 blocks of the fast path (waves 1..3)
struct SpecBuf {                       // LDS, 9216 B
  uint32_t ks[kSpecBlocks * 16];       // block b word w at ks[16 b + w] (b >= 1)
  uint32_t pw[kSpecPowers * 5];        // r^e (radix 2^26) at pw[5 (e - 1)]
};
struct SpecSlot {                      // LDS, 96 B
  uint32_t key[8];
  uint32_t nlo, nhi, valid, stamp;     // stamp: last use (LRU)
  uint32_t r[4], s[4];
  uint32_t nks, pmax, buf, pad;        // keystream blocks 1..nks, powers r^1..r^pmax, in bufs[buf]
};
// LDS words after the slots: the request broadcast (16 + the inline chunk
// count); the next nonce's
// block-0 words r0..3 (clamped), s0..3 and a valid flag; the fast path's
// wave-group counter and the spare table's index
constexpr uint32_t kResCmdWords = 20, kResPreWords = 16, kResSyncWords = 16;
__host__ __device__ constexpr size_t resident_lds_bytes() {
  return one_lds_bytes(kOneMaxAd, 65535u) + kSpecBufs * sizeof(SpecBuf) +
         kSpecSlots * sizeof(SpecSlot) + 4u * (kResCmdWords + kResPreWords + kResSyncWords);
}

__device__ __forceinline__ F26 pw_get(const SpecBuf *b, uint32_t e) {
  F26 f;
#pragma unroll
  for (int i = 0; i < 5; ++i) f.a[i] = b->pw[5u * (e - 1u) + i];
  return f;
}
__device__ __forceinline__ void pw_put(SpecBuf *b, uint32_t e, const F26 &f) {
#pragma unroll
  for (int i = 0; i < 5; ++i) b->pw[5u * (e - 1u) + i] = f.a[i];
}
// program-order LDS hand-off within ONE wave (no workgroup barrier)
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// LDS counter hand-offs between the waves of a group that do not all reach
// a workgroup barrier (the fast path: wave 0 speculates while waves 1..3
// serve the record): lane 0 of a wave arrives, any wave waits for a count
__device__ __forceinline__ void grp_arrive(uint32_t *c, uint32_t lane) {
  wave_sync_lds();  // every lane of the wave is here (lockstep on a GPU; the emulator's lanes are threads)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// one thread's arrival (from code only that thread runs)
__device__ __forceinline__ void grp_arrive1(uint32_t *c) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void grp_wait(uint32_t *c, uint32_t n) {
  while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < n)
    __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Block 0 of (key, nonce) on the quad of threads 0..3: pre[q] = r word q
// (clamped), pre[4 + q] = s word q, pre[8] = 1.  Called by all of wave 0
// (every quad computes, the first one stores: no divergence around the DPP).
__device__ __forceinline__ void spec_block0(uint32_t *pre, const uint32_t key[8], uint64_t nonce,
                                            uint32_t lane) {
  uint32_t kq[4];
  const uint32_t q = lane & 3u;
  chacha20_quad(key, q, 0u, (uint32_t)nonce, (uint32_t)(nonce >> 32), kq);
  if (lane < 4) {
    pre[q] = kq[0] & (q == 0 ? 0x0fffffffu : 0x0ffffffcu);
    pre[4 + q] = kq[1];
    if (q == 0) pre[8] = 1u;
  }
}

// Wave 0: the power ladder into b from r = pre[0..3] -- r^1..r^16, then
// r^32, r^48, .. by 16s up to 16 ceil(pmax / 16): one product per level,
// LDS ordered within the wave only (no workgroup barrier between levels).
__device__ void spec_ladder(SpecBuf *b, const uint32_t *pre, uint32_t pmax, uint32_t lane) {
  if (lane == 0) pw_put(b, 1u, to26(pre[0], pre[1], pre[2], pre[3], 0u));
  wave_sync_lds();
  // r^(l + i) = r^l r^i, i = 1 .. l: r^1 .. r^16
#pragma unroll 1
  for (uint32_t l = 1; l <= 8; l <<= 1) {
    if (lane < l) pw_put(b, l + lane + 1u, mul26(pw_get(b, l), pw_get(b, lane + 1u)));
    wave_sync_lds();
  }
  // r^(16 (l + i)) = r^(16 l) r^(16 i)
  const uint32_t m16 = (pmax + 15u) >> 4;
#pragma unroll 1
  for (uint32_t l = 1; l < m16; l <<= 1) {
    if (lane < l && l + lane + 1u <= m16)
      pw_put(b, 16u * (l + lane + 1u), mul26(pw_get(b, 16u * l), pw_get(b, 16u * (lane + 1u))));
    wave_sync_lds();
  }
}
// Waves 1..3: keystream blocks 1..nks of (key, nonce) into b, one per quad.
__device__ void spec_keystream(SpecBuf *b, const uint32_t key[8], uint64_t nonce, uint32_t nks,
                               uint32_t t) {
  const uint32_t wave = t >> 6, qd = (t - 64u) >> 2, wq0 = 16u * (wave - 1u);  // 48 quads
#pragma unroll 1
  for (uint32_t b0 = 1u + wq0; b0 <= nks; b0 += 48u) {  // wave-uniform trip count
    const uint32_t blk = b0 + (qd - wq0);
    uint32_t kq[4];
    chacha20_quad(key, t & 3u, blk, (uint32_t)nonce, (uint32_t)(nonce >> 32), kq);
    if (blk <= nks) {
#pragma unroll
      for (int r = 0; r < 4; ++r) b->ks[16u * blk + 4u * r + (t & 3u)] = kq[r];
    }
  }
}
// All threads: the powers that are not on the ladder, r^(16 a + c) = r^(16 a)
// r^c (one product each), then slot dst takes (key, nonce) with table b.
__device__ void spec_finish(SpecSlot *dst, uint32_t bi, SpecBuf *b, uint32_t *pre, uint32_t *sync,
                            const uint32_t key[8], uint64_t nonce, uint32_t stamp, uint32_t nks,
                            uint32_t pmax) {
  const uint32_t t = threadIdx.x;
  {
    const uint32_t e = t + 1u, hi = e >> 4, lo = e & 15u;
    if (e <= pmax && hi >= 1u && lo != 0u) pw_put(b, e, mul26(pw_get(b, 16u * hi), pw_get(b, lo)));
  }
  if (t == 0) {
    sync[1] = dst->buf;  // the slot's old table is the next spare
    dst->buf = bi;
    dst->nlo = (uint32_t)nonce;
    dst->nhi = (uint32_t)(nonce >> 32);
    dst->stamp = stamp;
    dst->nks = nks;
    dst->pmax = pmax;
  }
  if (t < 8) dst->key[t] = key[t];
  if (t < 4) {
    dst->r[t] = pre[t];
    dst->s[t] = pre[4 + t];
  }
  __syncthreads();
  if (t == 0) {
    dst->valid = 1u;
    pre[8] = 0u;
    sync[0] = 0u;  // the group counter, for the next request
  }
  __syncthreads();
}

// Sum of v over each row of 16 lanes (every lane of the row holds it): two
// quad_perm and two row_ror DPP adds, no LDS crossbar round trips.  The
// caller keeps the row sums below 2^32.
__device__ __forceinline__ uint32_t row_sum_dpp(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  return v;
}
__device__ __forceinline__ uint32_t rows_total(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// A speculated record (sp: (key, nonce)'s keystream blocks 1..nks and
// r^1..r^pmax in bufs[sp->buf]; the record has <= nks keystream blocks and
// P = na + nl + 1 <= min(pmax, 192) Poly1305 blocks).
//   waves 1..3: thread u = t - 64 < P takes block u (AD pieces, then
//     ciphertext pieces -- encrypt makes them here -- then the length
//     block) and computes (m_u + 2^128) r^(P-u); the products are summed per
//     wave by DPP (radix 2^26 limbs, renormalised after 16 terms) and the
//     three wave sums by thread 64, which adds s and writes / checks the tag.
//     Same result as the Horner chain of crypto_aead_write / crypto_aead_read
//     (monocypher.c:2858-2929): the sum IS that polynomial evaluated at r.
//     Their hand-offs are LDS counter waits (grp_*), not workgroup barriers,
//     and thread 64 raises the done word.
//   wave 0: waits for the record's DMA (it issued it at detection), lets
//     waves 1..3 go, then computes block 0 of nonce + 1 and its power ladder
//     into the spare table nb -- the speculation for the next record runs
//     while this one is served.
template <bool DECRYPT_T, bool RT = false>
__device__ void one_body_fast(const OneArgs &a, uint4 *lds, const SpecSlot *sp, const SpecBuf *cur,
                              SpecBuf *nb_, uint32_t pmax_next, uint32_t *pre, uint32_t *sync) {
  const bool DECRYPT = RT ? a.dec != 0u : DECRYPT_T;
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  const uint32_t L = a.len, A = a.ad_len;
  const uint32_t na = (A + 15u) >> 4, nl = (L + 15u) >> 4;
  const OneLayout lay = one_layout(A, L);
  uint8_t *base = a.base;
  const uint32_t s_tag = na + nl, s_ok = s_tag + 1, s_w = s_ok + 1;
  const uint32_t npc = na + nl + (DECRYPT ? 1u : 0u);
  uint32_t *gc = sync;  // 0 at entry
  if (wave == 0) {
    wait_vmem();  // the DMA this wave issued at detection
    grp_arrive(gc, lane);  // -> 1
    spec_block0(pre, a.key.w, a.nonce + 1u, lane);
    wave_sync_lds();
    spec_ladder(nb_, pre, pmax_next, lane);
    return;
  }
  const uint32_t u = t - 64u;
  grp_wait(gc, 1u);
  const uint32_t P = na + nl + 1u;
  F26 h;
#pragma unroll
  for (int i = 0; i < 5; ++i) h.a[i] = 0u;
  if (u < P) {
    uint4 m;
    if (u < na) {
      const uint32_t rem = A - 16u * u;
      m = mask_bytes(lds[u], rem >= 16u ? 16 : (int)rem);
    } else if (u < na + nl) {
      const uint32_t p = u - na, rem = L - 16u * p;
      const int nbytes = rem >= 16u ? 16 : (int)rem;
      const uint32_t *ks = cur->ks + 16u * (1u + (p >> 2)) + 4u * (p & 3u);
      const uint4 v = lds[na + p];
      if (!DECRYPT) {
        m = mask_bytes(make_uint4(v.x ^ ks[0], v.y ^ ks[1], v.z ^ ks[2], v.w ^ ks[3]), nbytes);
        lds[na + p] = m;  // ciphertext, zero padded
      } else {
        m = mask_bytes(v, nbytes);
      }
    } else {
      m = make_uint4(A, 0u, L, 0u);  // LE64(ad_len) || LE64(len)
    }
    h = mul26(to26(m.x, m.y, m.z, m.w, 1u), pw_get(cur, P - u));
  }
  // < 2^26 + 2^9 per term: a row's 16 terms fit in 32 bits, renormalised
  // before the four rows are added
#pragma unroll
  for (int i = 0; i < 5; ++i) h.a[i] = row_sum_dpp(h.a[i]);
  carry26(h);
#pragma unroll
  for (int i = 0; i < 5; ++i) h.a[i] = rows_total(h.a[i]);
  if (lane == 0) {
    lds[s_w + 2 * wave] = make_uint4(h.a[0], h.a[1], h.a[2], h.a[3]);
    lds[s_w + 2 * wave + 1] = make_uint4(h.a[4], 0u, 0u, 0u);
  }
  grp_arrive(gc, lane);  // -> 4
  if (t == 64) {
    grp_wait(gc, 4u);
    F26 H;
#pragma unroll
    for (int i = 0; i < 5; ++i) H.a[i] = 0u;
#pragma unroll
    for (uint32_t w = 1; w < kOneBlock / 64; ++w) {
      const uint4 v0 = lds[s_w + 2 * w], v1 = lds[s_w + 2 * w + 1];
      H.a[0] += v0.x; H.a[1] += v0.y; H.a[2] += v0.z; H.a[3] += v0.w; H.a[4] += v1.x;
    }
    carry26(H);
    carry26(H);
    Poly1305 p;
    from26(H, p.h0, p.h1, p.h2, p.h3, p.h4);
    p.s0 = sp->s[0]; p.s1 = sp->s[1]; p.s2 = sp->s[2]; p.s3 = sp->s[3];
    uint32_t tag[4];
    poly_final(p, tag);
    if (!DECRYPT) {
      lds[s_tag] = make_uint4(tag[0], tag[1], tag[2], tag[3]);
    } else {
      const uint4 w = lds[s_tag];
      lds[s_ok] = make_uint4((w.x ^ tag[0]) | (w.y ^ tag[1]) | (w.z ^ tag[2]) | (w.w ^ tag[3]), 0u,
                             0u, 0u);
    }
    grp_arrive1(gc);  // -> 5
  }
  grp_wait(gc, 5u);
  // LDS -> host image
  if (!DECRYPT) {
    if (u <= nl) {  // ct pieces, then the tag
      const uint4 v = lds[u < nl ? na + u : s_tag];
      const u32x4 w = {v.x, v.y, v.z, v.w};
      st_sys16(base, lay.out + 16ull * u, w);
    }
  } else {
    const bool ok = lds[s_ok].x == 0u;
    if (ok && u < nl) {  // verified: plaintext out
      const uint32_t rem = L - 16u * u;
      const uint32_t *ks = cur->ks + 16u * (1u + (u >> 2)) + 4u * (u & 3u);
      const uint4 v = lds[na + u];
      const uint4 o = mask_bytes(make_uint4(v.x ^ ks[0], v.y ^ ks[1], v.z ^ ks[2], v.w ^ ks[3]),
                                 rem >= 16u ? 16 : (int)rem);
      const u32x4 w = {o.x, o.y, o.z, o.w};
      st_sys16(base, lay.out + 16ull * u, w);
    }
    if (t == 64)
      __hip_atomic_store(reinterpret_cast<uint32_t *>(base) + 1,
                         ok ? NOISE_GPU_REC_OK : NOISE_GPU_REC_BAD_MAC, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // the request image zeroed (but for the seq words), every store drained,
  // then the done word (as one_finish, over waves 1..3)
  {
    const u32x4 z = {0u, 0u, 0u, 0u};
    if (!a.n_inl && u < npc) st_sys16(a.in_base, lay.ad + 16ull * u, z);
    req_wipe(a, u, kOneBlock - 64u);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  grp_arrive(gc, lane);  // -> 8
  if (t == 64) {
    grp_wait(gc, 8u);
    __hip_atomic_store(reinterpret_cast<uint32_t *>(a.base), a.seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// 16 bytes of the request image, bypassing the caches (the host rewrites it
// through the BAR behind the GPU's back)
__device__ __forceinline__ u32x4 ld_sys16(const uint8_t *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v) : "v"(p) : "memory");
  return v;
#else
  const volatile uint32_t *q = reinterpret_cast<const volatile uint32_t *>(p);
  u32x4 v = {q[0], q[1], q[2], q[3]};
  return v;
#endif
}

// chunks lane and 64 + lane of the request image in one go (two loads in
// flight, one wait)
__device__ __forceinline__ void ld_sys16x2(const uint8_t *p, u32x4 &c0, u32x4 &c1) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
               "global_load_dwordx4 %1, %2, off offset:1024 sc0 sc1\n\t"
               "s_waitcnt vmcnt(0)"
               : "=&v"(c0), "=&v"(c1) : "v"(p) : "memory");
#else
  c0 = ld_sys16(p);
  c1 = ld_sys16(p + 1024);
#endif
}

constexpr uint32_t kResSleepPolls = 4096u;  // empty polls before the wave backs off

// LDS: the staging image (one_lds_bytes(kOneMaxAd, 65535)), the
// speculation tables and slots, the request broadcast, the next block 0, the
// group counter
__global__ __launch_bounds__(kOneBlock) void k_aead_resident(uint8_t *req, uint8_t *base,
                                                             uint32_t last, uint64_t idle_ticks) {
#if defined(NOISE_HIP_EMU)
  uint4 *lds = reinterpret_cast<uint4 *>(emu::dyn_lds);  // tools/emu
#else
  extern __shared__ uint4 lds[];
#endif
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  const size_t stage = one_lds_bytes(kOneMaxAd, 65535u);
  SpecBuf *bufs = reinterpret_cast<SpecBuf *>(reinterpret_cast<uint8_t *>(lds) + stage);
  SpecSlot *slots = reinterpret_cast<SpecSlot *>(bufs + kSpecBufs);
  uint32_t *cmd = reinterpret_cast<uint32_t *>(slots + kSpecSlots);
  uint32_t *pre = cmd + kResCmdWords;
  uint32_t *sync = pre + kResPreWords;  // [0] group counter, [1] spare table
  if (t < kSpecSlots) {
    slots[t].valid = 0u;
    slots[t].buf = t;
  }
  if (t == 0) {
    pre[8] = 0u;
    sync[0] = 0u;
    sync[1] = kSpecSlots;
  }
  const OneRing *ring = reinterpret_cast<const OneRing *>(base + kOneRingOff);
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  uint32_t stamp = 0;
  __syncthreads();
  for (;;) {
    if (t < 64) {  // wave 0 polls chunks lane and 64 + lane (header: chunks 0..3)
      uint32_t ex = 0, polls = 0, n_inl = 0, dseq = 0;
      u32x4 c = {0u, 0u, 0u, 0u}, c1 = {0u, 0u, 0u, 0u};
      for (;;) {
        ld_sys16x2(req + 16u * lane, c, c1);
        // each chunk's seq, decoded with its own payload words (launchers.hpp
        // req_chunk_tag): a chunk that landed in part decodes to something
        // else.  Per lane and folded into the compares below -- no cross-lane
        // sum on the accept path.
        dseq = c.x ^ req_chunk_tag(lane, c.y, c.z, c.w);
        const uint32_t dseq1 = c1.x ^ req_chunk_tag(64u + lane, c1.y, c1.z, c1.w);
        const uint32_t seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)dseq);
        const uint64_t same = __ballot(lane < 4 && dseq == seq);
        if (seq != last && (same & 0xfull) == 0xfull) {
          // a complete header; an inline record must be complete too (every
          // chunk decodes to this seq), else poll again
          const uint32_t meta = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.y);
          n_inl = req_inline_chunks((meta >> 16) & 0x3fffu, meta & 0xffffu, (meta >> 30) & 1u);
          const bool need0 = lane >= 4u && lane - 4u < n_inl, need1 = 60u + lane < n_inl;
          if (__ballot((need0 && dseq != seq) || (need1 && dseq1 != seq)) == 0ull) {
            break;
          }
        }
        // a long-idle instance backs off after kResSleepPolls (4096, ~1 ms)
        // empty polls (s_sleep 32: ~2048 clocks, about one
        // more poll round trip, between polls): half the poll traffic and
        // issue slots; a request that follows the previous one within a few
        // ms is still seen at the full poll rate
        if (polls >= kResSleepPolls) __builtin_amdgcn_s_sleep(32);
        if ((++polls & 31u) == 0u) {
          // ONE decision for the wave (lane 0's).  On the GPU the stop word
          // is one load instruction and the clock a scalar read, so the lanes
          // agree anyway; the CPU emulator runs lanes as threads, which read
          // them at different times: a lane that saw the stop word (or the
          // idle deadline) flip first left the loop alone, the others waited
          // in the next __shfl for it for ever (emu_api's round-4 hang)
          const bool leave = __hip_atomic_load(&ring->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                             __builtin_amdgcn_s_memrealtime() - t_last > idle_ticks;
          if (__builtin_amdgcn_readfirstlane((int)leave)) {
            ex = 1;
            break;
          }
        }
      }
      if (!ex) {
        const uint32_t meta = (uint32_t)__shfl((int)c.y, 0);
        const uint32_t L = meta & 0xffffu, A = (meta >> 16) & 0x3fffu, dec = (meta >> 30) & 1u;
        if (n_inl) {  // the inline image: chunk k's 12 bytes -> LDS bytes [12k, 12k + 12)
          uint32_t *w = reinterpret_cast<uint32_t *>(lds);
          if (lane >= 4u && lane - 4u < n_inl) {
            const uint32_t k = lane - 4u;
            w[3u * k] = c.y; w[3u * k + 1u] = c.z; w[3u * k + 2u] = c.w;
          }
          if (60u + lane < n_inl) {
            const uint32_t k = 60u + lane;
            w[3u * k] = c1.y; w[3u * k + 1u] = c1.z; w[3u * k + 2u] = c1.w;
          }
        } else if (A <= kOneMaxAd) {  // issue the record's DMA at once (the bodies only wait for it)
          one_stage_in(req + kReqStageOff, one_layout(A, L),
                       ((A + 15u) >> 4) + ((L + 15u) >> 4) + dec, lds, lane, 64u);
        }
      }
      if (lane < 4) {
        cmd[4 * lane + 0] = c.x;
        cmd[4 * lane + 1] = c.y;
        cmd[4 * lane + 2] = c.z;
        cmd[4 * lane + 3] = c.w;
      }
      if (lane == 0) {
        cmd[0] = ex ? 0u : dseq;  // the decoded seq; 0: leave
        cmd[16] = n_inl;
      }
    }
    __syncthreads();
    const uint32_t n_inl = cmd[16];
    // chunk 0: seq, len | ad_len << 16 | decrypt << 30, nonce lo, hi;
    // chunks 1..3: seq + key words 0..2, 3..5, 6..7
    const uint32_t seq = cmd[0], meta = cmd[1];
    OneArgs a;
    a.nonce = ((uint64_t)cmd[3] << 32) | cmd[2];
    a.key.w[0] = cmd[5]; a.key.w[1] = cmd[6]; a.key.w[2] = cmd[7];
    a.key.w[3] = cmd[9]; a.key.w[4] = cmd[10]; a.key.w[5] = cmd[11];
    a.key.w[6] = cmd[13]; a.key.w[7] = cmd[14];
    const uint32_t spare = sync[1];
    __syncthreads();  // cmd is rewritten only after every thread has read it
    if (seq == 0u) break;
    a.base = base;
    a.in_base = req + kReqStageOff;
    a.req = req;
    a.n_inl = n_inl;
    a.len = meta & 0xffffu;
    a.ad_len = (meta >> 16) & 0x3fffu;
    a.seq = seq;
    a.wipe_in = 1u;
    a.staged = 1u;
    const uint32_t dec = (meta >> 30) & 1u;
    a.dec = dec;
    if (a.ad_len > kOneMaxAd || a.len > kResidentMaxLen) {  // the host never rings such a request
      a.ad_len = 0;
      a.len = 0;
      a.staged = 0u;
    }
    const uint32_t na = (a.ad_len + 15u) >> 4, nl = (a.len + 15u) >> 4;
    const uint32_t nb = (a.len + 63u) >> 6, P = na + nl + 1u;
    // a speculation slot for exactly this (key, nonce)?  and the slot the
    // next nonce goes to: the one holding this key, else the least recently
    // used one
    int hit = -1, dst = -1;
#pragma unroll
    for (uint32_t i = 0; i < kSpecSlots; ++i) {
      const SpecSlot &sp = slots[i];
      bool k = sp.valid != 0u;
#pragma unroll
      for (int w = 0; w < 8; ++w) k = k && sp.key[w] == a.key.w[w];
      if (k) dst = (int)i;
      if (k && sp.nlo == (uint32_t)a.nonce && sp.nhi == (uint32_t)(a.nonce >> 32) && nb <= sp.nks &&
          P <= sp.pmax)
        hit = (int)i;
    }
    if (dst < 0) dst = !slots[0].valid ? 0 : !slots[1].valid ? 1 : (slots[0].stamp <= slots[1].stamp ? 0 : 1);
    // the next speculation: as many keystream blocks as this record used (16
    // to 63) and powers for a record of this size (80, 128 or 192 blocks)
    const uint32_t nks = nb < 16u ? 16u : (nb > kSpecBlocks - 1u ? kSpecBlocks - 1u : nb);
    const uint32_t pmax = P <= 80u ? 80u : (P <= 128u ? 128u : kFastMaxBlocks);
    SpecBuf *nbuf = &bufs[spare];
    if (hit >= 0 && P <= kFastMaxBlocks) {
      // waves 1..3 serve, wave 0 starts the next speculation meanwhile
      one_body_fast<false, true>(a, lds, &slots[hit], &bufs[slots[hit].buf], nbuf, pmax, pre, sync);
      __syncthreads();
      if (wave != 0) spec_keystream(nbuf, a.key.w, a.nonce + 1u, nks, t);
    } else {
      one_body<false, true>(a, lds);
      if (wave == 0) {  // block 0 of the next nonce, then its ladder, beside the keystream
        spec_block0(pre, a.key.w, a.nonce + 1u, lane);
        wave_sync_lds();
        spec_ladder(nbuf, pre, pmax, lane);
      } else {
        spec_keystream(nbuf, a.key.w, a.nonce + 1u, nks, t);
      }
    }
    last = seq;
    __syncthreads();
    spec_finish(&slots[dst], spare, nbuf, pre, sync, a.key.w, a.nonce + 1u, ++stamp, nks, pmax);
#pragma unroll
    for (int i = 0; i < 8; ++i) a.key.w[i] = 0u;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  // leaving: no key or future keystream stays in this CU's LDS
  {
    uint32_t *w = reinterpret_cast<uint32_t *>(lds);
    const size_t nw = resident_lds_bytes() / 4;
    for (size_t i = t; i < nw; i += kOneBlock) w[i] = 0u;
  }
  __syncthreads();
  // gone: the host's unload hook waits for this word (done line, offset 8)
  if (t == 0) {
    __threadfence_system();
    __hip_atomic_store(reinterpret_cast<uint32_t *>(base + 8), 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

constexpr int kMaxAttrDev = 64;


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
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)resident_lds_bytes());
    attr_err[dev] = r;
  });
  return attr_err[dev];
}

hipError_t launch_aead_resident(uint8_t *d_req, uint8_t *d_base, uint32_t last, uint32_t idle_us,
                                hipStream_t stream) {
  const hipError_t e = one_attr();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_aead_resident, dim3(1), dim3(kOneBlock), resident_lds_bytes(), stream, d_req,
                     d_base, last, (uint64_t)idle_us * 100ull);  // s_memrealtime: 100 MHz
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
  a.in_base = d_base;
  a.len = len;
  a.ad_len = ad_len;
  a.seq = seq;
  a.wipe_in = 0u;
  a.staged = 0u;
  a.req = nullptr;
  a.n_inl = 0u;
  a.dec = decrypt ? 1u : 0u;
  const size_t lds = one_lds_bytes(ad_len, len);
  if (decrypt)
    hipLaunchKernelGGL((k_aead_one<true>), dim3(1), dim3(kOneBlock), lds, stream, a);
  else
    hipLaunchKernelGGL((k_aead_one<false>), dim3(1), dim3(kOneBlock), lds, stream, a);
  for (int i = 0; i < 8; ++i) a.key.w[i] = 0u;
  return hipGetLastError();
}

}  // namespace noise_amd
