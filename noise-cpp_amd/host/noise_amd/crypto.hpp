// noise_amd/crypto.hpp -- host-side primitives of the Noise handshake
// (Noise_*_25519_ChaChaPoly_BLAKE2b): BLAKE2b (RFC 7693), HMAC-BLAKE2b and the
// Noise HKDF (Noise rev34 §4.3), X25519 (RFC 7748), OS randomness.
//
// These replace the reference's handshake-side calls into Monocypher
// (crypto_blake2b*, monocypher.c:451-652; crypto_x25519, 1546-1563) and its
// noise.cpp adapters hash / hmac_hash / hkdf / dh / generate_keypair
// (noise.cpp:164-177, 283-374).  They are latency-bound, per-handshake host
// work; the transport AEAD is the GPU's.
#pragma once
#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace noise::crypto {

constexpr std::size_t kHashLen = 64;   // BLAKE2b-512
constexpr std::size_t kBlockLen = 128;
constexpr std::size_t kDhLen = 32;

using Hash = std::array<std::uint8_t, kHashLen>;
using Key32 = std::array<std::uint8_t, 32>;

// Incremental BLAKE2b, unkeyed, 1..64-byte digest.
class Blake2b {
 public:
  explicit Blake2b(std::size_t outlen = kHashLen);
  void update(const std::uint8_t *p, std::size_t n);
  void final(std::uint8_t *out);  // writes outlen bytes
 private:
  void compress(bool last);
  std::uint64_t h_[8];
  std::uint64_t t_[2] = {0, 0};
  std::uint8_t buf_[kBlockLen];
  std::size_t fill_ = 0, outlen_;
};

Hash blake2b(const std::uint8_t *p, std::size_t n);
// HMAC-BLAKE2b (RFC 2104, 128-byte block) over the concatenation a || b
Hash hmac(const std::uint8_t *key, std::size_t key_len, const std::uint8_t *a,
          std::size_t a_len, const std::uint8_t *b = nullptr, std::size_t b_len = 0);
// Noise HKDF(chaining_key, input_key_material, num_outputs = 2 or 3)
void hkdf(const Hash &ck, const std::uint8_t *ikm, std::size_t ikm_len, Hash *out1,
          Hash *out2, Hash *out3 = nullptr);

// X25519(scalar, u) -> u-coordinate (RFC 7748 §5, clamped scalar)
Key32 x25519(const Key32 &scalar, const Key32 &u);
Key32 x25519_base(const Key32 &scalar);  // X25519(scalar, 9)

// OS randomness (getrandom / /dev/urandom); throws std::runtime_error
void random_bytes(std::uint8_t *p, std::size_t n);

// constant-time compare / wipe (monocypher.c:144-167 semantics)
bool verify(const std::uint8_t *a, const std::uint8_t *b, std::size_t n);
void wipe(void *p, std::size_t n);

}  // namespace noise::crypto
