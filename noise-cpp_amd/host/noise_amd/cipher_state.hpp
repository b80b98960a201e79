// noise_amd/cipher_state.hpp -- drop-in noise::CipherState backed by the
// MI355X AEAD engine (include/noise_gpu.h).
//
// Surface and layout are those of the reference's class (noise.h:99-115):
// private `std::array<uint8_t,32> k; uint64_t n;`, the same public members
// with the same signatures and the same exceptions:
//   std::out_of_range("Nonce limit has been exceeded!")  n == 2^64-2
//                                                        (noise.cpp:398-400)
//   std::invalid_argument("Invalid MAC")                 (noise.cpp:246/275)
// plus batch members (non-virtual, no layout change) for device-resident and
// multi-record use.  Integration: INTEGRATION.md.
//
// Deliberate, documented deviations from the literal reference:
//  * has_key() follows the Noise spec (key present <=> k != 0^32).  The
//    reference returns crypto_verify32(k, 0) == 0 (noise.cpp:386-389),
//    i.e. true only for the all-zero key, which makes every post-handshake
//    encrypt_with_ad a silent plaintext pass-through.
//  * decrypt of fewer than 16 bytes throws invalid_argument (the reference
//    underflows, noise.cpp:257).
// Kept as in the reference: the nonce limit at 2^64-2 (equality test),
// n advancing even when the MAC check fails (noise.cpp:421), rekey at
// nonce 2^64-2 (noise.cpp:435), the destructor wiping k and setting
// n = UINT64_MAX (noise.cpp:376-379).
#pragma once
#include <array>
#include <concepts>
#include <cstddef>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <vector>

namespace noise {

#ifndef NOISE_STL_CONTAINER_DEFINED
#define NOISE_STL_CONTAINER_DEFINED
template <typename T>
concept STLContainer = requires(T container) {
  typename T::iterator;
  { container.data() } -> std::same_as<typename T::value_type *>;
  { container.size() } -> std::same_as<std::size_t>;
};
#endif

// The reference's exported free functions (noise.cpp:202-224 encrypt,
// 254-281 decrypt; `T` symbols of its library, declared nowhere public), with
// the same signature -- so the same mangled name -- on the GPU engine:
//   encrypt: in_out grows by 16 (ct || tag, noise.cpp:206) under the nonce
//            0^32 || LE64(n) (noise.cpp:207-215), AD = *ad when present;
//   decrypt: the tag is checked first; on failure in_out is left untouched
//            and std::invalid_argument("Invalid MAC") is thrown (noise.cpp:
//            269-276), else it shrinks by 16 (noise.cpp:280);
//   both wipe the caller's key k after use, as the reference does
//            (crypto_wipe(k), noise.cpp:221-223 / 277-279).
// Deviations, as for CipherState: decrypt of fewer than 16 bytes throws
// invalid_argument("Invalid MAC") (the reference underflows, noise.cpp:257);
// an all-zero k is "no key" (noise_gpu.h) and throws invalid_argument;
// no gfx950 device -> std::runtime_error.  No nonce-limit check here: that
// rule is CipherState's (noise.cpp:398), the free functions have none.
void encrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out);
void decrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out);

class CipherState {
private:
  // zero-initialised (the reference leaves both indeterminate under its
  // defaulted constructor, noise.h:101-105): a fresh CipherState has no key
  std::array<std::uint8_t, 32> k{};
  std::uint64_t n = 0;

  void encrypt_raw(const std::uint8_t *ad, std::size_t ad_len,
                   std::vector<std::uint8_t> &plaintext);
  void decrypt_raw(const std::uint8_t *ad, std::size_t ad_len,
                   std::vector<std::uint8_t> &ciphertext);

public:
  CipherState() = default;
  ~CipherState();
  void initialize_key(const std::array<std::uint8_t, 32> &key);
  [[nodiscard]] bool has_key() const;
  void set_nonce(const std::uint64_t &nonce);
  template <STLContainer T> void encrypt_with_ad(T &ad, T &plaintext);
  void encrypt_with_ad(std::vector<std::uint8_t> &plaintext);
  template <STLContainer T> void decrypt_with_ad(T &ad, T &ciphertext);
  void decrypt_with_ad(std::vector<std::uint8_t> &ciphertext);
  void rekey();

  // ---- batch extensions (not in the reference surface) -----------------
  // Current nonce (the reference keeps n private and has no getter).
  [[nodiscard]] std::uint64_t nonce() const { return n; }
  // The key, for handing a session to a device-side batch (the key table of
  // noise_gpu_*_records / noise::transport::Batcher).
  [[nodiscard]] const std::array<std::uint8_t, 32> &key_material() const { return k; }

  // Encrypt every message in order with nonces n, n+1, ... exactly as a
  // loop of encrypt_with_ad would (each grows by 16).  Stops with
  // out_of_range at the nonce limit after encrypting the records before it.
  void encrypt_batch(std::vector<std::vector<std::uint8_t>> &messages);
  // Decrypt in order.  n advances for every message (as the per-record
  // path does, failures included).  Messages whose tag fails are left
  // unchanged and flagged in `ok` (if given); after the whole batch one
  // invalid_argument("Invalid MAC") is thrown if any failed.
  void decrypt_batch(std::vector<std::vector<std::uint8_t>> &messages,
                     std::vector<std::uint8_t> *ok = nullptr);

  // Device-resident uniform batch of `count` records of `len` bytes:
  // d_in records (stride in_stride) -> d_out ct||tag records (stride
  // out_stride), nonces n..n+count-1, asynchronous on `stream`
  // (hipStream_t).  Applies the nonce limit like encrypt_batch.
  void encrypt_device(const std::uint8_t *d_in, std::uint64_t in_stride,
                      std::uint8_t *d_out, std::uint64_t out_stride,
                      std::uint32_t len, std::uint64_t count,
                      void *stream = nullptr);
  // Device-resident decrypt; per-record status in d_status (0 ok, 1 bad
  // MAC), n += count.  Failures are reported through d_status only (the
  // call is asynchronous).
  void decrypt_device(const std::uint8_t *d_in, std::uint64_t in_stride,
                      std::uint8_t *d_out, std::uint64_t out_stride,
                      std::uint32_t len, std::uint8_t *d_status,
                      std::uint64_t count, void *stream = nullptr);
};

template <STLContainer T>
void CipherState::encrypt_with_ad(T &ad, T &plaintext) {
  if (!has_key()) return;
  std::vector<std::uint8_t> buf(plaintext.begin(), plaintext.end());
  encrypt_raw(reinterpret_cast<const std::uint8_t *>(ad.data()), ad.size(), buf);
  plaintext.resize(buf.size());
  std::copy(buf.begin(), buf.end(), plaintext.begin());
}

template <STLContainer T>
void CipherState::decrypt_with_ad(T &ad, T &ciphertext) {
  if (!has_key()) return;
  std::vector<std::uint8_t> buf(ciphertext.begin(), ciphertext.end());
  decrypt_raw(reinterpret_cast<const std::uint8_t *>(ad.data()), ad.size(), buf);
  ciphertext.resize(buf.size());
  std::copy(buf.begin(), buf.end(), ciphertext.begin());
}

// The vector instantiation (the only one the reference links) works in place.
template <>
inline void CipherState::encrypt_with_ad<std::vector<std::uint8_t>>(
    std::vector<std::uint8_t> &ad, std::vector<std::uint8_t> &plaintext) {
  if (!has_key()) return;
  encrypt_raw(ad.data(), ad.size(), plaintext);
}
template <>
inline void CipherState::decrypt_with_ad<std::vector<std::uint8_t>>(
    std::vector<std::uint8_t> &ad, std::vector<std::uint8_t> &ciphertext) {
  if (!has_key()) return;
  decrypt_raw(ad.data(), ad.size(), ciphertext);
}

}  // namespace noise
