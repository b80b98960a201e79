// Microbenchmark: VALU issue throughput of the integer instructions the
// ChaCha20 / Poly1305 kernels are built from (gfx950). Each kernel runs ITERS
// iterations of 8 independent instruction streams per lane (inline asm so the
// exact opcode is issued), 2048 blocks x 256 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 32768

#define BODY8(INSN)                                                          \
  asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c));                            \
  asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));

#define K32(NAME, INSN)                                                      \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                       \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, \
             a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;             \
    uint32_t b = seed * 3 + threadIdx.x, c = seed ^ 0x55;                    \
    for (int i = 0; i < ITERS; ++i) { BODY8(INSN) }                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                             \
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                               \
  }

K32(k_add, "v_add_u32 %0, %0, %1")
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %0, 20")
K32(k_perm, "v_perm_b32 %0, %0, %1, %2")
K32(k_add3, "v_add3_u32 %0, %0, %1, %2")
K32(k_xad, "v_xad_u32 %0, %0, %1, %2")
K32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
K32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_add_e64, "v_add_u32_e64 %0, %0, %1")
K32(k_add_lit, "v_add_u32_e32 %0, 0x12345, %0")
K32(k_align3, "v_alignbit_b32 %0, %1, %2, 20")
K32(k_xor_sdwa, "v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")
K32(k_lshl, "v_lshlrev_b32_e32 %0, 7, %0")
K32(k_or3, "v_or3_b32 %0, %0, %1, %2")
K32(k_addc, "v_addc_co_u32 %0, vcc, %0, %1, vcc")

// 64-bit accumulate forms
#define BODY8_64(INSN)                                                       \
  asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c) : "vcc");                    \
  asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c) : "vcc");

#define K64(NAME, INSN)                                                      \
  __global__ void NAME(uint64_t *out, uint32_t seed) {                       \
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, \
             a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;             \
    uint32_t b = seed * 3 + threadIdx.x, c = seed ^ 0x55;                    \
    for (int i = 0; i < ITERS; ++i) { BODY8_64(INSN) }                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                             \
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                               \
  }
K64(k_mad64, "v_mad_u64_u32 %0, vcc, %1, %2, %0")
K64(k_fma64, "v_fma_f64 %0, %0, %0, %0")
K64(k_lshl64, "v_lshlrev_b64 %0, 3, %0")


__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define QR(a, b, c, d) a += b; d = rotl(d ^ a, 16); c += d; b = rotl(b ^ c, 12); a += b; d = rotl(d ^ a, 8); c += d; b = rotl(b ^ c, 7);
// 16 independent words as 4 independent QR chains; counts 12*8 = 96 ops per iteration
__global__ void k_chacha(uint32_t *out, uint32_t seed) {
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * (i + 1) ^ seed;
  for (int i = 0; i < ITERS / 12; ++i) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_clock(unsigned long long *out) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) asm volatile("v_add_u32 %0, %0, 1" : "+v"(a));
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = r1 - r0; }
  if (a == 12345678) out[0] = 0;
}


__global__ void k_chacha2(uint32_t *out, uint32_t seed) {
  uint32_t x[16], y[16];
  for (int i = 0; i < 16; ++i) { x[i] = threadIdx.x * (i + 1) ^ seed; y[i] = x[i] * 3 + i; }
  for (int i = 0; i < ITERS / 24; ++i) {
    QR(x[0], x[4], x[8], x[12]) QR(y[0], y[4], y[8], y[12]) QR(x[1], x[5], x[9], x[13]) QR(y[1], y[5], y[9], y[13])
    QR(x[2], x[6], x[10], x[14]) QR(y[2], y[6], y[10], y[14]) QR(x[3], x[7], x[11], x[15]) QR(y[3], y[7], y[11], y[15])
    QR(x[0], x[5], x[10], x[15]) QR(y[0], y[5], y[10], y[15]) QR(x[1], x[6], x[11], x[12]) QR(y[1], y[6], y[11], y[12])
    QR(x[2], x[7], x[8], x[13]) QR(y[2], y[7], y[8], y[13]) QR(x[3], x[4], x[9], x[14]) QR(y[3], y[4], y[9], y[14])
  }
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r ^= x[i] ^ y[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
#define CHAIN1(INSN) asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c));
__global__ void k_add_dep(uint32_t *out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, b = seed * 3 + threadIdx.x, c = seed ^ 0x55;
  for (int i = 0; i < ITERS; ++i) { CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1")
                                    CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1") CHAIN1("v_add_u32 %0, %0, %1") }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
__global__ void k_align_dep(uint32_t *out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, b = seed * 3 + threadIdx.x, c = seed ^ 0x55;
  for (int i = 0; i < ITERS; ++i) { CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20")
                                    CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20") CHAIN1("v_alignbit_b32 %0, %0, %0, 20") }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
// alternate fast/slow independent
__global__ void k_alt(uint32_t *out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed * 3 + threadIdx.x, c = seed ^ 0x55;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b)); asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a1));
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(b)); asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a3));
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(b)); asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a5));
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(b)); asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename T>
static void run(const char *name, void (*k)(T *, uint32_t)) {
  const int blocks = 2048, threads = 256;
  T *out;
  hipMalloc(&out, sizeof(T) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double insts = 5.0 * blocks * threads * (double)ITERS * 8; if ((void*)k == (void*)k_chacha2) insts = 5.0 * blocks * threads * (double)(ITERS / 24) * 192; if ((void*)k == (void*)k_chacha) insts = 5.0 * blocks * threads * (double)(ITERS / 12) * 96;  // lane-ops
  double rate = insts / (ms * 1e-3);
  // lane-ops per clock per CU at 2.4 GHz, 256 CUs
  printf("%-12s %8.3f ms  %7.2f T lane-op/s  %6.1f lane-op/clk/CU(@2.4GHz)\n",
         name, ms, rate / 1e12, rate / 256 / 2.4e9);
  hipFree(out);
}

int main() {
  { unsigned long long *o; hipMalloc(&o, 2048*16); hipLaunchKernelGGL(k_clock, dim3(2048), dim3(256), 0, 0, o); hipDeviceSynchronize();
    unsigned long long h[4096]; hipMemcpy(h, o, 2048*16, hipMemcpyDeviceToHost);
    double s = 0; for (int i = 0; i < 2048; ++i) s += (double)h[2*i] / h[2*i+1] * 100.0; printf("in-kernel clock ~ %.0f MHz\n", s / 2048); }
  run<uint32_t>("chacha_mix", k_chacha);
  run<uint32_t>("chacha_x2", k_chacha2);
  run<uint32_t>("add_dep", k_add_dep);
  run<uint32_t>("align_dep", k_align_dep);
  run<uint32_t>("alt_add_align", k_alt);
  run<uint32_t>("add_u32", k_add);
  run<uint32_t>("xor_b32", k_xor);
  run<uint32_t>("alignbit", k_alignbit);
  run<uint32_t>("perm_b32", k_perm);
  run<uint32_t>("add3_u32", k_add3);
  run<uint32_t>("xad_u32", k_xad);
  run<uint32_t>("mul_lo_u32", k_mul_lo);
  run<uint32_t>("mul_hi_u32", k_mul_hi);
  run<uint32_t>("mad_u32_u24", k_mad24);
  run<uint32_t>("mul_hi_u24", k_mulhi24);
  run<uint32_t>("addc_co", k_addc);
  run<uint32_t>("add_e64", k_add_e64);
  run<uint32_t>("add_lit", k_add_lit);
  run<uint32_t>("align3", k_align3);
  run<uint32_t>("xor_sdwa", k_xor_sdwa);
  run<uint32_t>("lshl_e32", k_lshl);
  run<uint32_t>("or3", k_or3);
  run<uint64_t>("mad_u64_u32", k_mad64);
  run<uint64_t>("fma_f64", k_fma64);
  run<uint64_t>("lshl_b64", k_lshl64);
  return 0;
}
