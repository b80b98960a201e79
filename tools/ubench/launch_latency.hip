// launch_latency.hip -- where the time of a one-record GPU call goes on
// MI355X (the CipherState::encrypt_with_ad latency path, single_kernels.hip).
// Each variant is timed 2000 times; medians in microseconds.
//   sync_empty      empty kernel + hipStreamSynchronize
//   flag_empty      kernel stores a done word to host-mapped memory; host polls it
//   flag_read1k     + the kernel first reads 1 KiB of host-mapped memory (64 lanes x 16 B)
//   flag_rw1k       + writes 1 KiB back to host-mapped memory before the done word
//   copy_path       hipMemcpyAsync H2D 1 KiB + empty kernel + D2H 1 KiB + sync
//   flag_alu        flag_rw1k + ~1000 dependent VALU ops per lane (one ChaCha block)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                          \
    }                                                                    \
  } while (0)

__global__ void k_empty() {}

template <int MODE>
__global__ __launch_bounds__(64) void k_flag(uint8_t *base, uint32_t seq, uint32_t iters) {
  __shared__ uint4 lds[64];
  const uint32_t t = threadIdx.x;
  uint4 v = make_uint4(t, 0, 0, 0);
  if (MODE >= 1) v = reinterpret_cast<const uint4 *>(base + 1024)[t];
  if (MODE >= 3) {
    uint32_t a = v.x, b = v.y, c = v.z, d = v.w;
    for (uint32_t i = 0; i < iters; ++i) {
      a += b; d = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 16);
      c += d; b = __builtin_amdgcn_alignbit(b ^ c, b ^ c, 20);
    }
    v = make_uint4(a, b, c, d);
  }
  lds[t] = v;
  __syncthreads();
  if (MODE >= 2) reinterpret_cast<uint4 *>(base + 4096)[t] = lds[63 - t];
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) __hip_atomic_store(reinterpret_cast<uint32_t *>(base), seq, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median(std::vector<double> &v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint8_t *h = nullptr, *d = nullptr, *dev = nullptr, *hp = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void **>(&h), 1 << 16, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0));
  CHECK(hipHostMalloc(reinterpret_cast<void **>(&hp), 1 << 16, hipHostMallocDefault));
  CHECK(hipMalloc(reinterpret_cast<void **>(&dev), 1 << 16));
  std::memset(h, 0, 1 << 16);
  const int N = 2000;
  uint32_t seq = 0;
  auto flag_run = [&](auto kern, uint32_t iters) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i) {
      const uint32_t s = ++seq;
      const auto a = clk::now();
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, st, d, s, iters);
      while (*reinterpret_cast<volatile uint32_t *>(h) != s) {
      }
      const auto b = clk::now();
      if (i >= 50) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    (void)hipStreamSynchronize(st);
    return median(t);
  };
  std::vector<double> t;
  for (int i = 0; i < N + 50; ++i) {
    const auto a = clk::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    (void)hipStreamSynchronize(st);
    const auto b = clk::now();
    if (i >= 50) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::printf("sync_empty   %7.2f us\n", median(t));
  std::printf("flag_empty   %7.2f us\n", flag_run(k_flag<0>, 0));
  std::printf("flag_read1k  %7.2f us\n", flag_run(k_flag<1>, 0));
  std::printf("flag_rw1k    %7.2f us\n", flag_run(k_flag<2>, 0));
  std::printf("flag_alu250  %7.2f us  (~1000 dependent VALU ops per lane)\n", flag_run(k_flag<3>, 125));
  std::printf("flag_alu1000 %7.2f us  (~4000 dependent VALU ops per lane)\n", flag_run(k_flag<3>, 500));
  t.clear();
  for (int i = 0; i < N + 50; ++i) {
    const auto a = clk::now();
    (void)hipMemcpyAsync(dev, hp, 1024, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    (void)hipMemcpyAsync(hp, dev, 1040, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    const auto b = clk::now();
    if (i >= 50) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::printf("copy_path    %7.2f us\n", median(t));
  // host-side cost of the launch call alone
  t.clear();
  for (int i = 0; i < N; ++i) {
    const auto a = clk::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    const auto b = clk::now();
    t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    if (i % 64 == 63) (void)hipStreamSynchronize(st);
  }
  (void)hipStreamSynchronize(st);
  std::printf("launch_call  %7.2f us  (host time inside hipLaunchKernelGGL)\n", median(t));
  return 0;
}
