// Ablation of the tile kernel (tile_kernel.hpp): full vs no-HBM vs no-Poly,
// 2^20 x 1 KiB encrypt, contiguous records.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "tile_kernel.hpp"
using namespace noise_amd;
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
    for (int r = 0; r < 20; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    printf("%-12s %8.3f ms  %7.1f GB/s alg (2064 B/record)\n", name, ms, R * 2064.0 / (ms * 1e-3) / 1e9);
  };
  const dim3 g(R / 64), b(64);
  TileArgs ea{}, da{};
  ea.key = key; ea.in = in; ea.in_stride = L; ea.out = out; ea.out_stride = L + 16; ea.nrec = R;
  da = ea; da.in = out; da.in_stride = L + 16; da.out = in; da.out_stride = L; da.status = out;
  for (int rep = 0; rep < 2; ++rep) {
    timeit("full", [&] { hipLaunchKernelGGL((k_aead_tile<false, 1024, true, kTileUniform, 0>), g, b, 0, 0, ea); });
    timeit("no_hbm", [&] { hipLaunchKernelGGL((k_aead_tile<false, 1024, true, kTileUniform, 1>), g, b, 0, 0, ea); });
    timeit("no_poly", [&] { hipLaunchKernelGGL((k_aead_tile<false, 1024, true, kTileUniform, 2>), g, b, 0, 0, ea); });
    timeit("dec_full", [&] { hipLaunchKernelGGL((k_aead_tile<true, 1024, true, kTileUniform, 0>), g, b, 0, 0, da); });
  }
  return 0;
}
