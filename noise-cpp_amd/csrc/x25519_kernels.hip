// x25519_kernels.hip -- batched X25519 on gfx950 (SURVEY.md §8(f) rank 4:
// DH for mass handshakes).  Replaces, for many sessions at once, the
// reference's noise::dh -> crypto_x25519 (noise.cpp:172-177,
// monocypher.c:1546-1563); written from RFC 7748 §5 (clamped scalar,
// Montgomery ladder, a24 = 121665).  One lane = one scalar multiplication
// (x25519_device.hpp); public keys (points == NULL) take the fixed-base
// edwards25519 table path instead of the ladder.
#include "x25519_device.hpp"
#include "launchers.hpp"

namespace noise_amd {

// out[i] = X25519(scalars[i], points ? points[i] : 9); 32 bytes each
__global__ __launch_bounds__(64) void k_x25519(const u32x4 *__restrict__ scalars,
                                               const u32x4 *__restrict__ points,
                                               u32x4 *__restrict__ out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], w[8];
  {
    const u32x4 a = scalars[2 * i], b = scalars[2 * i + 1];
    k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
  }
  if (points) {
    uint32_t u[8];
    const u32x4 a = points[2 * i], b = points[2 * i + 1];
    u[0] = a.x; u[1] = a.y; u[2] = a.z; u[3] = a.w; u[4] = b.x; u[5] = b.y; u[6] = b.z; u[7] = b.w;
    x25519::scalarmult(w, k, u);
  } else {  // public keys: the fixed-base table path (wave-uniform branch)
    x25519::base_scalarmult(w, k);
  }
  out[2 * i] = u32x4{w[0], w[1], w[2], w[3]};
  out[2 * i + 1] = u32x4{w[4], w[5], w[6], w[7]};
}
hipError_t launch_x25519(const uint8_t *scalars, const uint8_t *points, uint8_t *out, uint64_t n,
                         hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_x25519, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, stream,
                     reinterpret_cast<const u32x4 *>(scalars),
                     reinterpret_cast<const u32x4 *>(points), reinterpret_cast<u32x4 *>(out), n);
  return hipGetLastError();
}

}  // namespace noise_amd
