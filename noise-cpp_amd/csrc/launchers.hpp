// launchers.hpp -- internal interface between the C-ABI layer
// (noise_gpu_api.hip) and the kernels (aead_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "noise_gpu.h"

namespace noise_amd {

hipError_t launch_aead_uniform(bool decrypt, const uint32_t key[8],
                               uint64_t nonce0, const uint8_t *in,
                               uint64_t in_stride, uint8_t *out,
                               uint64_t out_stride, uint32_t len,
                               const uint8_t *ad, uint64_t ad_stride,
                               uint32_t ad_len, uint8_t *status, uint64_t nrec,
                               hipStream_t stream);

hipError_t launch_aead_records(bool decrypt, const uint8_t *keys,
                               uint32_t nkeys, const noise_gpu_record *recs,
                               uint64_t nrec, const uint8_t *in, uint8_t *out,
                               const uint8_t *ad, uint8_t *status,
                               hipStream_t stream);

bool sessions_supported(uint32_t len, const void *in, uint64_t in_stride,
                        const void *out, uint64_t out_stride);

hipError_t launch_aead_sessions(bool decrypt, const uint8_t *keys,
                                uint32_t nkeys, const uint32_t *key_idx,
                                const uint64_t *nonces, const uint8_t *in,
                                uint64_t in_stride, uint8_t *out,
                                uint64_t out_stride, uint32_t len,
                                uint8_t *status, uint64_t nrec,
                                hipStream_t stream);

hipError_t launch_rekey(uint8_t *keys, uint64_t nkeys, hipStream_t stream);

hipError_t launch_x25519(const uint8_t *scalars, const uint8_t *points,
                         uint8_t *out, uint64_t n, hipStream_t stream);

hipError_t launch_fill_synthetic(uint8_t *dst, uint64_t offset,
                                 uint64_t nbytes, uint64_t seed,
                                 hipStream_t stream);

}  // namespace noise_amd
