// Ablation of the lane-per-record AEAD kernel: where do the 4 ms go?
//   full       : the product device code (encrypt, 2^20 x 1 KiB)
//   compute    : same code, all lanes read records from a 256 KiB L2-resident
//                window, no ciphertext stores (tag only)
//   mem_lane   : lane-per-record access pattern (64 B per lane per chunk),
//                XOR with a constant, no ChaCha / Poly
//   mem_quad   : 4 lanes per record, 256 B per record per step
//   copy       : fully coalesced dwordx4 copy of the same bytes
#include <hip/hip_runtime.h>
#include <cstdio>
#include "chachapoly_device.hpp"
using namespace noise_amd;

struct KeyArg { uint32_t w[8]; };

template <bool COMPUTE_ONLY>
__global__ __launch_bounds__(256) void k_full(KeyArg key, const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrec) return;
  uint32_t k[8];
  for (int j = 0; j < 8; ++j) k[j] = key.w[j];
  if (!COMPUTE_ONLY) {
    aead_record<false, true>(k, i, in + i * len, out + i * (len + 16), len, nullptr, 0);
  } else {
    // read from a 256-record window, write only the tag
    const uint8_t *src = in + (i & 255) * len;
    const uint32_t n_lo = (uint32_t)i, n_hi = 0;
    Poly1305 p;
    { uint32_t otk[16]; chacha20_block(k, 0u, n_lo, n_hi, otk); poly_init(p, otk); }
    for (uint32_t c = 0; c < len / 64; ++c) {
      uint32_t ks[16];
      chacha20_block(k, 1u + c, n_lo, n_hi, ks);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = load16<true>(src + 64 * c + 16 * q, 16);
        poly_block(p, v.x ^ ks[4 * q], v.y ^ ks[4 * q + 1], v.z ^ ks[4 * q + 2], v.w ^ ks[4 * q + 3]);
      }
    }
    poly_block(p, 0, 0, len, 0);
    uint32_t tag[4];
    poly_final(p, tag);
    store16<true>(out + i * (len + 16) + len, make_uint4(tag[0], tag[1], tag[2], tag[3]), 16);
  }
}

__global__ __launch_bounds__(256) void k_mem_lane(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrec) return;
  const uint8_t *src = in + i * len;
  uint8_t *dst = out + i * (len + 16);
  uint32_t acc = (uint32_t)i;
  for (uint32_t c = 0; c < len / 64; ++c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = load16<true>(src + 64 * c + 16 * q, 16);
      v.x ^= acc; acc += v.y;
      store16<true>(dst + 64 * c + 16 * q, v, 16);
    }
  }
  store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}

// 4 lanes per record; lane j handles chunks j, j+4, j+8, j+12
__global__ __launch_bounds__(256) void k_mem_quad(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t i = t >> 2;
  const uint32_t j = t & 3;
  if (i >= nrec) return;
  const uint8_t *src = in + i * len;
  uint8_t *dst = out + i * (len + 16);
  uint32_t acc = (uint32_t)i;
  for (uint32_t c = j; c < len / 64; c += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = load16<true>(src + 64 * c + 16 * q, 16);
      v.x ^= acc; acc += v.y;
      store16<true>(dst + 64 * c + 16 * q, v, 16);
    }
  }
  if (j == 0) store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}


// lane-per-record, chunk order rotated by lane (start chunk = lane % 16)
__global__ __launch_bounds__(256) void k_mem_lane_rot(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrec) return;
  const uint8_t *src = in + i * len;
  uint8_t *dst = out + i * (len + 16);
  uint32_t acc = (uint32_t)i;
  const uint32_t nch = len / 64, s = threadIdx.x % nch;
  for (uint32_t t = 0; t < nch; ++t) {
    uint32_t c = t + s; if (c >= nch) c -= nch;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = load16<true>(src + 64 * c + 16 * q, 16);
      v.x ^= acc; acc += v.y;
      store16<true>(dst + 64 * c + 16 * q, v, 16);
    }
  }
  store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}
// lane-per-record, 128 B per step (two chunks, 8 loads in flight)
__global__ __launch_bounds__(256) void k_mem_lane_x2(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrec) return;
  const uint8_t *src = in + i * len;
  uint8_t *dst = out + i * (len + 16);
  uint32_t acc = (uint32_t)i;
  for (uint32_t c = 0; c < len / 128; ++c) {
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = load16<true>(src + 128 * c + 16 * q, 16);
#pragma unroll
    for (int q = 0; q < 8; ++q) { v[q].x ^= acc; acc += v[q].y; store16<true>(dst + 128 * c + 16 * q, v[q], 16); }
  }
  store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}
// records at a 1040-byte input stride too (no power-of-two stride anywhere)
__global__ __launch_bounds__(256) void k_mem_lane_1040(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrec) return;
  const uint8_t *src = in + i * (len + 16);
  uint8_t *dst = out + i * (len + 16);
  uint32_t acc = (uint32_t)i;
  for (uint32_t c = 0; c < len / 64; ++c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = load16<true>(src + 64 * c + 16 * q, 16);
      v.x ^= acc; acc += v.y;
      store16<true>(dst + 64 * c + 16 * q, v, 16);
    }
  }
  store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}
// coalesced whole-record staging: 64-thread WG, 64 records, LDS row stride 1040
__global__ __launch_bounds__(64) void k_mem_lds(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  __shared__ uint4 lds[64 * 65];
  const uint64_t r0 = (uint64_t)blockIdx.x * 64;
  const uint32_t l = threadIdx.x;
  const uint4 *src = reinterpret_cast<const uint4 *>(in + r0 * len);
  for (int k = 0; k < 64; ++k) lds[k * 65 + l] = src[k * 64 + l];  // record k, piece l
  __syncthreads();
  uint32_t acc = (uint32_t)(r0 + l);
  uint8_t *dst = out + (r0 + l) * (len + 16);
  for (int p = 0; p < 64; ++p) {
    uint4 v = lds[l * 65 + p];
    v.x ^= acc; acc += v.y;
    store16<true>(dst + 16 * p, v, 16);
  }
  store16<true>(dst + len, make_uint4(acc, 0, 0, 0), 16);
}


// SEG-byte contiguous segments per instruction: lanes grouped SEG/16 per
// segment; segment k of instruction q = record (q * (64*16/SEG) + k), bytes
// [SEG*t, SEG*(t+1)) of the record at step t.  A wave owns 64 records.
template <int SEG>
__global__ __launch_bounds__(256) void k_mem_seg(const uint8_t *in, uint8_t *out, uint32_t len, uint64_t nrec) {
  constexpr int LPS = SEG / 16;          // lanes per segment
  constexpr int SPI = 64 / LPS;          // segments (records) per instruction
  constexpr int NI = 64 / SPI;           // instructions to cover 64 records
  const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const uint32_t l = threadIdx.x & 63;
  const uint64_t r0 = wave * 64;
  if (r0 >= nrec) return;
  uint32_t acc = l;
  for (uint32_t t = 0; t < len / SEG; ++t) {
    uint4 v[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const uint64_t r = r0 + q * SPI + l / LPS;
      v[q] = load16<true>(in + r * len + SEG * t + 16 * (l % LPS), 16);
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const uint64_t r = r0 + q * SPI + l / LPS;
      v[q].x ^= acc; acc += v[q].y;
      store16<true>(out + r * (len + 16) + SEG * t + 16 * (l % LPS), v[q], 16);
    }
  }
  if (l < 64) store16<true>(out + (r0 + l) * (len + 16) + len, make_uint4(acc, 0, 0, 0), 16);
}

__global__ __launch_bounds__(256) void k_copy(const uint4 *in, uint4 *out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    uint4 v = in[i];
    v.x ^= 1;
    out[i] = v;
  }
}

int main() {
  const uint64_t R = 1 << 20;
  const uint32_t L = 1024;
  uint8_t *in, *out;
  (void)hipMalloc(&in, R * L);
  (void)hipMalloc(&out, R * (L + 16));
  (void)hipMemset(in, 0x5a, R * L);
  KeyArg key;
  for (int j = 0; j < 8; ++j) key.w[j] = 0x03020100u + 0x04040404u * j;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timeit = [&](const char *name, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-10s %8.3f ms  %7.1f GB/s (2064 B/record)\n", name, ms, R * 2064.0 / (ms * 1e-3) / 1e9);
  };
  const dim3 g((R + 255) / 256), b(256);
  if (0) timeit("full", [&] { hipLaunchKernelGGL((k_full<false>), g, b, 0, 0, key, in, out, L, R); });
  if (0) timeit("compute", [&] { hipLaunchKernelGGL((k_full<true>), g, b, 0, 0, key, in, out, L, R); });
  timeit("mem_lane", [&] { hipLaunchKernelGGL(k_mem_lane, g, b, 0, 0, in, out, L, R); });
  timeit("mem_quad", [&] { hipLaunchKernelGGL(k_mem_quad, dim3(g.x * 4), b, 0, 0, in, out, L, R); });
  if (0) timeit("lane_rot", [&] { hipLaunchKernelGGL(k_mem_lane_rot, g, b, 0, 0, in, out, L, R); });
  timeit("lane_x2", [&] { hipLaunchKernelGGL(k_mem_lane_x2, g, b, 0, 0, in, out, L, R); });
  uint8_t *in2; (void)hipMalloc(&in2, R * (L + 16));
  if (0) timeit("lane_1040", [&] { hipLaunchKernelGGL(k_mem_lane_1040, g, b, 0, 0, in2, out, L, R); });
  timeit("lds_stage", [&] { hipLaunchKernelGGL(k_mem_lds, dim3(R / 64), dim3(64), 0, 0, in, out, L, R); });
  timeit("seg64", [&] { hipLaunchKernelGGL(k_mem_seg<64>, g, b, 0, 0, in, out, L, R); });
  timeit("seg128", [&] { hipLaunchKernelGGL(k_mem_seg<128>, g, b, 0, 0, in, out, L, R); });
  timeit("seg256", [&] { hipLaunchKernelGGL(k_mem_seg<256>, g, b, 0, 0, in, out, L, R); });
  timeit("seg1024", [&] { hipLaunchKernelGGL(k_mem_seg<1024>, g, b, 0, 0, in, out, L, R); });
  timeit("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(4096), b, 0, 0, (const uint4 *)in, (uint4 *)out, R * L / 16); });
  return 0;
}
