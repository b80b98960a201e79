// sessions_kernels.hip -- many-session batches (BASELINE config 3): the
// LDS-staged tile kernel with per-record key rows and nonces (KEYED).
// Kept in its own translation unit: co-compiling the KEYED and uniform
// instantiations in one TU trips a gfx950 codegen error in ROCm 7.2
// ("Illegal instruction detected: Operand has incorrect register class" on
// an LDS address-space check).
#include "chachapoly_device.hpp"
#include "launchers.hpp"
#include "tile_kernel.hpp"

namespace noise_amd {

bool sessions_supported(uint32_t len, const void *in, uint64_t in_stride,
                        const void *out, uint64_t out_stride) {
  const bool vec = ((reinterpret_cast<uintptr_t>(in) |
                     reinterpret_cast<uintptr_t>(out) | in_stride |
                     out_stride | len) & 15u) == 0;
  switch (len) {
    case 64: case 128: case 192: case 256: case 512: case 1024: case 2048:
    case 4096: case 8192: case 16384:
      return vec;
    default:
      return false;
  }
}

hipError_t launch_aead_sessions(bool decrypt, const uint8_t *keys,
                                uint32_t nkeys, const uint32_t *key_idx,
                                const uint64_t *nonces, const uint8_t *in,
                                uint64_t in_stride, uint8_t *out,
                                uint64_t out_stride, uint32_t len,
                                uint8_t *status, uint64_t nrec,
                                hipStream_t stream) {
  if (nrec == 0) return hipSuccess;
  TileArgs ta{};
  ta.in = in;
  ta.in_stride = in_stride;
  ta.out = out;
  ta.out_stride = out_stride;
  ta.status = status;
  ta.nrec = nrec;
  ta.in_place = in == out;
  ta.keys = keys;
  ta.nkeys = nkeys;
  ta.key_idx = key_idx;
  ta.nonces = nonces;
  const dim3 gt((unsigned)((nrec + 63) / 64)), bt(64);
  const bool contig = decrypt ? (in_stride == (uint64_t)len + 16 && out_stride == len)
                              : (in_stride == len && out_stride == (uint64_t)len + 16);
#define NOISE_SESS_LAUNCH(DEC, LEN, CONTIG)                                    \
    hipLaunchKernelGGL((k_aead_tile<DEC, LEN, CONTIG, kTileSessions>), gt, bt, 0, stream, ta)
#define NOISE_SESS_CASE(LEN)                                                   \
    case LEN:                                                                  \
      if (decrypt) {                                                           \
        if (contig) NOISE_SESS_LAUNCH(true, LEN, true);                        \
        else NOISE_SESS_LAUNCH(true, LEN, false);                              \
      } else {                                                                 \
        if (contig) NOISE_SESS_LAUNCH(false, LEN, true);                       \
        else NOISE_SESS_LAUNCH(false, LEN, false);                             \
      }                                                                        \
      return hipGetLastError();
  switch (len) {
    NOISE_SESS_CASE(64)
    NOISE_SESS_CASE(128)
    NOISE_SESS_CASE(192)
    NOISE_SESS_CASE(256)
    NOISE_SESS_CASE(512)
    NOISE_SESS_CASE(1024)
    NOISE_SESS_CASE(2048)
    NOISE_SESS_CASE(4096)
    NOISE_SESS_CASE(8192)
    NOISE_SESS_CASE(16384)
    default:
      return hipErrorInvalidValue;
  }
#undef NOISE_SESS_CASE
#undef NOISE_SESS_LAUNCH
}

}  // namespace noise_amd
