// one_timing.hip -- where the single-record latency kernel (k_aead_one,
// single_kernels.hip) spends its time: the product source built with
// NOISE_ONE_TIMING, so thread 0 stamps s_memrealtime (100 MHz) at the phase
// boundaries of one_body into the staging's done line.  Per record size and
// direction, the median over 60 calls of each phase and of the host's wall
// time from launch to the done word.
//   one_timing   -> one line per (len, direction)
#define NOISE_ONE_TIMING 1
#include "single_kernels.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace noise_amd;

int main() {
  const OneLayout big = one_layout(0, 65535);
  uint8_t *h = nullptr, *d = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), big.total + 4096,
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0) != hipSuccess) return 1;
  std::memset(h, 0, big.total + 4096);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  uint32_t key[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  uint32_t seq = 0;
  std::vector<uint8_t> ctag;
  std::printf("# us: [0] entry->DMA issued+keystream  [1] DMA wait+XOR+sync  [2] Poly1305+tag  "
              "[3] stores  [4] fence+sync  | kernel total | host wall (launch->done)\n");
  for (uint32_t L : {64u, 1024u, 4096u, 16384u, 65519u}) {
    const OneLayout lay = one_layout(0, L);
    for (int dec = 0; dec < 2; ++dec) {
      std::vector<double> ph[5], tot, wall;
      for (int it = 0; it < 60; ++it) {
        if (dec) {  // decrypt what the last encrypt produced: ct || tag
          std::memcpy(h + lay.in, ctag.data(), L);
          std::memcpy(h + lay.tag, ctag.data() + L, 16);
        } else {
          for (uint32_t i = 0; i < L; ++i) h[lay.in + i] = (uint8_t)(i * 7 + it);
        }
        const uint32_t s = ++seq;
        const auto t0 = std::chrono::steady_clock::now();
        if (launch_aead_one(dec != 0, key, 77, d, L, 0, s, st) != hipSuccess) return 2;
        volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(h);
        while (*done != s) {
        }
        const auto t1 = std::chrono::steady_clock::now();
        (void)hipStreamSynchronize(st);
        const uint64_t *ts = reinterpret_cast<const uint64_t *>(h + kOneTsOff);
        for (int i = 0; i < 5; ++i) ph[i].push_back((ts[i + 1] - ts[i]) * 0.01);
        tot.push_back((ts[5] - ts[0]) * 0.01);
        wall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        if (!dec) {
          ctag.assign(h + lay.out, h + lay.out + L);
          ctag.insert(ctag.end(), h + lay.out + ((L + 15) & ~15u), h + lay.out + ((L + 15) & ~15u) + 16);
        }
        if (dec && reinterpret_cast<volatile uint32_t *>(h)[1] != 0) {
          std::printf("decrypt failed\n");
          return 3;
        }
      }
      auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
      };
      std::printf("L %5u %s: %.2f %.2f %.2f %.2f %.2f | %.2f | %.2f\n", L, dec ? "dec" : "enc",
                  med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]), med(tot), med(wall));
    }
  }
  return 0;
}
