// Characterise gfx950 VALU issue cost of instruction mixes (cycles per
// wave-instruction per SIMD), varying waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 16384
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define QR(a, b, c, d) a += b; d = rotl(d ^ a, 16); c += d; b = rotl(b ^ c, 12); a += b; d = rotl(d ^ a, 8); c += d; b = rotl(b ^ c, 7);
__global__ void k_chacha(uint32_t *out, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * (i + 1) ^ seed;
  for (int i = 0; i < ITERS / 8; ++i) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// rotations by 16 / 8 through v_perm_b32 instead of alignbit
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x01000302u); }
__device__ __forceinline__ uint32_t rot8(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x02010003u); }
#define QRP(a, b, c, d) a += b; d = rot16(d ^ a); c += d; b = rotl(b ^ c, 12); a += b; d = rot8(d ^ a); c += d; b = rotl(b ^ c, 7);
__global__ void k_chacha_perm(uint32_t *out, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * (i + 1) ^ seed;
  for (int i = 0; i < ITERS / 8; ++i) {
    QRP(x[0], x[4], x[8], x[12]) QRP(x[1], x[5], x[9], x[13]) QRP(x[2], x[6], x[10], x[14]) QRP(x[3], x[7], x[11], x[15])
    QRP(x[0], x[5], x[10], x[15]) QRP(x[1], x[6], x[11], x[12]) QRP(x[2], x[7], x[8], x[13]) QRP(x[3], x[4], x[9], x[14])
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// only adds+xors of chacha (rotations removed) -- to price the fast part
#define QRN(a, b, c, d) a += b; d = (d ^ a); c += d; b = (b ^ c); a += b; d = (d ^ a); c += d; b = (b ^ c);
__global__ void k_chacha_norot(uint32_t *out, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * (i + 1) ^ seed;
  for (int i = 0; i < ITERS / 8; ++i) {
    QRN(x[0], x[4], x[8], x[12]) QRN(x[1], x[5], x[9], x[13]) QRN(x[2], x[6], x[10], x[14]) QRN(x[3], x[7], x[11], x[15])
    QRN(x[0], x[5], x[10], x[15]) QRN(x[1], x[6], x[11], x[12]) QRN(x[2], x[7], x[8], x[13]) QRN(x[3], x[4], x[9], x[14])
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// rotations only (4 independent chains x 4)
__global__ void k_rot_only(uint32_t *out, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * (i + 1) ^ seed;
  for (int i = 0; i < ITERS / 8; ++i) {
#pragma unroll
    for (int j = 0; j < 32; ++j) x[j & 15] = rotl(x[j & 15], 7 + (j & 3));
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static double clock_ghz = 2.2;
static void run(const char *name, void (*k)(uint32_t *, uint32_t), double inst_per_iter, int waves_per_simd) {
  const int threads = 256;
  const int blocks = 256 * waves_per_simd;  // 4 waves/block, 4 SIMDs/CU
  uint32_t *out;
  (void)hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double wave_insts = 5.0 * blocks * (threads / 64) * (double)(ITERS / 8) * inst_per_iter;
  double per_simd = wave_insts / 1024.0;
  double cyc = ms * 1e-3 * clock_ghz * 1e9;
  printf("%-14s waves/SIMD=%d  %8.3f ms  %.2f cyc per wave-inst per SIMD\n", name, waves_per_simd, ms, cyc / per_simd);
  (void)hipFree(out);
}
int main() {
  for (int w : {1, 2, 4, 8}) {
    run("chacha", k_chacha, 96, w);
    run("chacha_perm", k_chacha_perm, 96, w);
    run("chacha_norot", k_chacha_norot, 64, w);
    run("rot_only", k_rot_only, 32, w);
  }
  return 0;
}
