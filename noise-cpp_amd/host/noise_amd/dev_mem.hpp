// dev_mem.hpp -- stream-ordered device allocations for the engine's own
// buffers that grow or go away while the device may be busy (internal).
//
// hipFree (and hipHostFree) on ROCm wait for every stream of the device before
// they return.  A resident latency instance (noise_gpu_set_resident) occupies
// its stream until it idles out, so with steady single-record traffic on one
// thread, a hipFree on another thread -- a records scratch that grows, a
// Pipeline key table that doubles -- would wait for a gap in that traffic,
// possibly for ever.  hipMallocAsync / hipFreeAsync order the allocation and
// the free on ONE stream instead: the free happens once the work queued on that
// stream before it has run, and nothing else is waited for.  A device without
// memory pools falls back to hipMalloc / hipFree (the answer is kept per
// device, so an allocation and its free always take the same path).
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstddef>

namespace noise_amd {

inline bool dev_pools(int dev) {
#if defined(NOISE_NO_MEMPOOL)
  (void)dev;
  return false;
#endif
  constexpr int kMaxDev = 64;
  static std::atomic<int> known[kMaxDev];  // 0 unknown, 1 pools, 2 none
  if (dev < 0 || dev >= kMaxDev) return false;
  int v = known[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    int a = 0;
    const bool ok = hipDeviceGetAttribute(&a, hipDeviceAttributeMemoryPoolsSupported, dev) ==
                        hipSuccess && a != 0;
    v = ok ? 1 : 2;
    known[dev].store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

// bytes of device memory on the current device, usable by work queued on
// `stream` after this call (and, after an event, by other streams)
inline hipError_t dev_alloc(void **p, size_t bytes, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev_pools(dev)) return hipMallocAsync(p, bytes, stream);
  return hipMalloc(p, bytes);
}

// zero `bytes` of p (secret hygiene) and free it once the work queued on
// `stream` so far has run; `stream` must order after every use of p
inline hipError_t dev_wipe_free(void *p, size_t bytes, hipStream_t stream) {
  if (!p) return hipSuccess;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (bytes) e = hipMemsetAsync(p, 0, bytes, stream);
  hipError_t e2;
  if (dev_pools(dev)) {
    e2 = hipFreeAsync(p, stream);
  } else {
    e2 = hipStreamSynchronize(stream);
    const hipError_t e3 = hipFree(p);
    if (e2 == hipSuccess) e2 = e3;
  }
  return e != hipSuccess ? e : e2;
}

// dev_alloc / dev_wipe_free work on the CURRENT device (their pool choice
// is per device): an owner bound to one device (a Pipeline) holds this guard
// around them, so the allocation, its free and every HIP call in between
// target the owner's device whatever device the calling thread has current
struct DeviceGuard {
  int prev = -1, want;
  explicit DeviceGuard(int dev) : want(dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != want) (void)hipSetDevice(want);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;
};

}  // namespace noise_amd
