// doorbell_probe.hip -- where should a resident kernel's doorbell live?
// Host <-> GPU ping-pong round trips with the flag the GPU polls in
//   (a) host-mapped coherent pinned memory (hipHostMalloc Mapped|Coherent),
//   (b) fine-grained device memory (hipExtMallocWithFlags Finegrained), if
//       the host can store to it (probed with a caught SIGSEGV / SIGBUS first),
// and the reply always in host-mapped memory.  One workgroup, one lane
// polling; the kernel leaves after `iters` round trips or a 2 s timeout
// (s_memrealtime), whichever comes first.
//   doorbell_probe   -> lines "mode ... rt_us median / p10 / p90"
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// flag: the doorbell (host writes i); reply: the GPU writes i back
__global__ void k_pong(uint32_t *flag, uint32_t *reply, int iters, int use_sc1_load) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t last = 0;
  for (int n = 0; n < iters;) {
    const uint32_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != last) {
      last = v;
      __hip_atomic_store(reply, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ++n;
      continue;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;  // 2 s
    (void)use_sc1_load;
  }
}

static sigjmp_buf g_jb;
static void on_fault(int) { siglongjmp(g_jb, 1); }
// a host store to p: 1 if it lands, 0 if it faults (SIGSEGV / SIGBUS caught
// in-process; no fork, nothing else touched)
static int can_host_store(void *p) {
  struct sigaction sa {}, o1, o2;
  sa.sa_handler = on_fault;
  sigaction(SIGSEGV, &sa, &o1);
  sigaction(SIGBUS, &sa, &o2);
  int ok = 0;
  if (sigsetjmp(g_jb, 1) == 0) {
    volatile uint32_t *q = static_cast<volatile uint32_t *>(p);
    q[0] = 0x1234u;
    ok = q[0] == 0x1234u;
  }
  sigaction(SIGSEGV, &o1, nullptr);
  sigaction(SIGBUS, &o2, nullptr);
  return ok;
}

// flag in host memory or device memory behind the BAR (write-combined on
// the host: sfence after the store pushes it out)
static void run(const char *name, uint32_t *hflag, uint32_t *dflag, uint32_t *hreply,
                uint32_t *dreply, bool fence = false) {
  const int iters = 2000;
  volatile uint32_t *f = hflag, *r = hreply;
  *f = 0;
  *r = 0;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, s, dflag, dreply, iters, 0);
  std::vector<double> rt;
  for (uint32_t i = 1; i <= (uint32_t)iters; ++i) {
    const auto a = std::chrono::steady_clock::now();
    *f = i;
    if (fence) _mm_sfence();
    uint64_t spins = 0;
    while (*r != i && ++spins < 400000000ull) {
    }
    const auto b = std::chrono::steady_clock::now();
    if (*r != i) {
      std::printf("%s: no reply at %u\n", name, i);
      break;
    }
    rt.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  if (rt.empty()) return;
  std::sort(rt.begin(), rt.end());
  std::printf("%-34s rt_us median %.2f  p10 %.2f  p90 %.2f  (n=%zu)\n", name, rt[rt.size() / 2],
              rt[rt.size() / 10], rt[rt.size() * 9 / 10], rt.size());
}

int main() {
  uint32_t *hreply = nullptr, *dreply = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&hreply), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dreply), hreply, 0));
  // (a) host pinned flag
  uint32_t *hflag = nullptr, *dflag = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&hflag), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dflag), hflag, 0));
  run("host-mapped coherent flag", hflag, dflag, hreply, dreply);
  // (b) fine-grained VRAM, host store + sfence
  uint32_t *fg = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void **>(&fg), 4096, hipDeviceMallocFinegrained) ==
      hipSuccess) {
    if (can_host_store(fg)) run("fine-grained VRAM flag + sfence", fg, fg, hreply, dreply, true);
    else std::printf("fine-grained VRAM: host store faults\n");
  } else {
    std::printf("fine-grained VRAM: allocation failed\n");
  }
  // (c) coarse VRAM (plain hipMalloc), host store + sfence, GPU sc1 polls
  uint32_t *cg = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(&cg), 4096) == hipSuccess) {
    if (can_host_store(cg)) run("hipMalloc VRAM flag + sfence", cg, cg, hreply, dreply, true);
    else std::printf("hipMalloc VRAM: host store faults\n");
  }
  // host memory again, to compare in the same run
  run("host-mapped coherent flag (again)", hflag, dflag, hreply, dreply);
  return 0;
}
