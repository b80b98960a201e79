// blake2b_device.hpp -- BLAKE2b-512 (RFC 7693), HMAC-BLAKE2b and the Noise
// HKDF (rev34 §4.3) as per-lane device functions for the batched handshake
// kernels (handshake_kernels.hip).  Replaces, for many sessions at once, the
// reference's noise::hash / hmac_hash / hkdf (noise.cpp:283-374) over
// Monocypher's crypto_blake2b (monocypher.c:451-652); unkeyed, 64-byte
// output, as the reference's HASH (HASHLEN 64, BLOCKLEN 128).
//
// gfx950 mapping: a 64-bit word is two VGPRs; the 64-bit adds are
// v_add_co/v_addc pairs, rotr 32 is a register rename, rotr 24/16/63 two
// v_alignbit each -- ~26 VALU instructions per G, ~2.5 K per compression.
// Every value a handshake hashes is either in registers (h, ck, keys, DH
// results) or a short message in HBM, so there is no buffering layer: the
// callers assemble whole 128-byte blocks and call b2_compress from as few
// sites as possible (each site is a ~10 KB unrolled body).
#pragma once
#include "chachapoly_device.hpp"

namespace noise_amd {
namespace b2 {

__device__ __forceinline__ uint64_t iv(int i) {
  switch (i) {
    case 0: return 0x6a09e667f3bcc908ull;
    case 1: return 0xbb67ae8584caa73bull;
    case 2: return 0x3c6ef372fe94f82bull;
    case 3: return 0xa54ff53a5f1d36f1ull;
    case 4: return 0x510e527fade682d1ull;
    case 5: return 0x9b05688c2b3e6c1full;
    case 6: return 0x1f83d9abfb41bd6bull;
    default: return 0x5be0cd19137e2179ull;
  }
}

// message schedule (RFC 7693 §2.7); rounds 10 and 11 reuse rows 0 and 1
constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
};

__device__ __forceinline__ uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

#define NOISE_B2_G(a, b, c, d, x, y)  \
  a = a + b + (x);                    \
  d = rotr(d ^ a, 32);                \
  c = c + d;                          \
  b = rotr(b ^ c, 24);                \
  a = a + b + (y);                    \
  d = rotr(d ^ a, 16);                \
  c = c + d;                          \
  b = rotr(b ^ c, 63);

// h <- F(h, m, t, last): one BLAKE2b compression (RFC 7693 §3.2), byte
// counter t < 2^64 (a Noise message is <= 65535 bytes)
__device__ __forceinline__ void compress(uint64_t h[8], const uint64_t m[16], uint64_t t,
                                         bool last) {
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = h[i];
    v[i + 8] = iv(i);
  }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    const uint8_t *s = kSigma[r % 10];
    NOISE_B2_G(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
    NOISE_B2_G(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
    NOISE_B2_G(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
    NOISE_B2_G(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
    NOISE_B2_G(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
    NOISE_B2_G(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
    NOISE_B2_G(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
    NOISE_B2_G(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}
#undef NOISE_B2_G

// parameter block of an unkeyed 64-byte digest: h0 ^= 0x01010040
__device__ __forceinline__ void init(uint64_t h[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = iv(i);
  h[0] ^= 0x01010040ull;
}

__device__ __forceinline__ uint64_t w64(const uint32_t *w, int i) {
  return (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// Little-endian 8-byte word of p[off .. off+8) clipped to [0, len), zero
// padded.  ALIGNED: p + off is 8-byte aligned.
__device__ __forceinline__ uint64_t load_word(const uint8_t *p, int64_t off, int64_t len,
                                              bool aligned) {
  if (off >= len) return 0;
  if (aligned && off + 8 <= len) return *reinterpret_cast<const uint64_t *>(p + off);
  uint64_t x = 0;
  const int64_t n = len - off < 8 ? len - off : 8;
  for (int64_t b = 0; b < n; ++b) x |= (uint64_t)p[off + b] << (8 * b);
  return x;
}

// MixHash from memory: h <- BLAKE2b(h || data[0..len)) (noise.cpp:474-486).
// The first block is h (64 B, registers) and data[0..64); then 128-byte
// blocks of data.  One compression site.
__device__ __forceinline__ void mix_hash_mem(uint32_t hw[16], const uint8_t *data, int64_t len) {
  uint64_t st[8];
  init(st);
  const int64_t total = 64 + len;
  const int64_t nb = total <= 128 ? 1 : (total + 127) / 128;
  const bool aligned = (reinterpret_cast<uintptr_t>(data) & 7u) == 0;
#pragma unroll 1
  for (int64_t b = 0; b < nb; ++b) {
    uint64_t m[16];
    if (b == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = w64(hw, j);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[8 + j] = load_word(data, 8 * j, len, aligned);
    } else {
      const int64_t base = 128 * b - 64;
#pragma unroll
      for (int j = 0; j < 16; ++j) m[j] = load_word(data, base + 8 * j, len, aligned);
    }
    const bool last = b == nb - 1;
    compress(st, m, last ? (uint64_t)total : (uint64_t)(128 * (b + 1)), last);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hw[2 * j] = (uint32_t)st[j];
    hw[2 * j + 1] = (uint32_t)(st[j] >> 32);
  }
}

// MixHash of a 32-byte value in registers: one compression
__device__ __forceinline__ void mix_hash32(uint32_t hw[16], const uint32_t d[8]) {
  uint64_t st[8], m[16];
  init(st);
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = w64(hw, j);
#pragma unroll
  for (int j = 0; j < 4; ++j) m[8 + j] = w64(d, j);
#pragma unroll
  for (int j = 12; j < 16; ++j) m[j] = 0;
  compress(st, m, 96, true);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hw[2 * j] = (uint32_t)st[j];
    hw[2 * j + 1] = (uint32_t)(st[j] >> 32);
  }
}

// MixHash of a 64-byte value in registers (MixKeyAndHash's temp_h): one
// full block, h || d
__device__ __forceinline__ void mix_hash64(uint32_t hw[16], const uint32_t d[16]) {
  uint64_t st[8], m[16];
  init(st);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = w64(hw, j);
    m[8 + j] = w64(d, j);
  }
  compress(st, m, 128, true);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hw[2 * j] = (uint32_t)st[j];
    hw[2 * j + 1] = (uint32_t)(st[j] >> 32);
  }
}

// HKDF(ck, ikm) of Noise rev34 §4.3 over HMAC-BLAKE2b (RFC 2104, block 128):
//   temp = HMAC(ck, ikm); o1 = HMAC(temp, 0x01); o2 = HMAC(temp, o1 || 0x02);
//   o3 = HMAC(temp, o2 || 0x03)                    (noise.cpp:293-374)
// ikm is 32 bytes (DH output, public key, psk) or empty (ilen 0: the inner
// message of HMAC(ck, empty) is the ipad block alone).  The ipad / opad states
// of a key are computed once and shared by the outputs under it:
// 4 + 2 + 2*nout compressions (one fewer for an empty ikm).  Two compression sites (inner, outer), both in
// one loop: step 0 is HMAC(ck, ikm), steps 1..nout the outputs.
__device__ __forceinline__ void hkdf(const uint32_t ck[16], const uint32_t ikm[8], int ilen,
                                     int nout, uint32_t o1[16], uint32_t o2[16],
                                     uint32_t o3[16]) {
  uint64_t key[8], si[8], so[8], prev[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    key[j] = w64(ck, j);
    prev[j] = 0;
  }
#pragma unroll 1
  for (int step = 0; step <= nout; ++step) {
    if (step <= 1) {  // key states for ck (step 0) and temp (step 1)
      uint64_t m[16];
#pragma unroll 1
      for (int pad = 0; pad < 2; ++pad) {
        const uint64_t x = pad ? 0x5c5c5c5c5c5c5c5cull : 0x3636363636363636ull;
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = key[j] ^ x;
#pragma unroll
        for (int j = 8; j < 16; ++j) m[j] = x;
        uint64_t s[8];
        init(s);
        // HMAC(ck, empty) (Split): the ipad block is the whole inner message
        compress(s, m, 128, pad == 0 && step == 0 && ilen == 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (pad) so[j] = s[j];
          else si[j] = s[j];
        }
      }
    }
    // inner block: step 0 -> ikm; step k -> o_{k-1} (64 B, none for k=1) || k
    uint64_t m[16];
    uint64_t dlen;
    if (step == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = ilen ? w64(ikm, j) : 0ull;
#pragma unroll
      for (int j = 4; j < 16; ++j) m[j] = 0;
      dlen = (uint64_t)ilen;
    } else if (step == 1) {
      m[0] = 1;
#pragma unroll
      for (int j = 1; j < 16; ++j) m[j] = 0;
      dlen = 1;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = prev[j];
      m[8] = (uint64_t)step;
#pragma unroll
      for (int j = 9; j < 16; ++j) m[j] = 0;
      dlen = 65;
    }
    uint64_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = si[j];
    if (step != 0 || ilen != 0) compress(x, m, 128 + dlen, true);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = x[j];
      m[8 + j] = 0;
      x[j] = so[j];
    }
    compress(x, m, 192, true);
    if (step == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) key[j] = x[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) prev[j] = x[j];
      // uniform branches: the outputs stay in registers
      if (step == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { o1[2 * j] = (uint32_t)x[j]; o1[2 * j + 1] = (uint32_t)(x[j] >> 32); }
      } else if (step == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { o2[2 * j] = (uint32_t)x[j]; o2[2 * j + 1] = (uint32_t)(x[j] >> 32); }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { o3[2 * j] = (uint32_t)x[j]; o3[2 * j + 1] = (uint32_t)(x[j] >> 32); }
      }
    }
  }
}

}  // namespace b2
}  // namespace noise_amd
