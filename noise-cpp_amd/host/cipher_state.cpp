// cipher_state.cpp -- noise::CipherState over the C ABI (include/noise_gpu.h).
// Host-side rules only (nonce bookkeeping, key presence, exceptions); every
// byte of ChaCha20-Poly1305 is computed by the gfx950 kernels.
// Reference behaviour mirrored: noise.cpp:376-439.
#include "noise_amd/cipher_state.hpp"

#include <algorithm>
#include <cstring>
#include <limits>
#include <string>

#include "noise_gpu.h"

namespace noise {
namespace {

constexpr std::uint64_t kNonceLimit = std::numeric_limits<std::uint64_t>::max() - 1;

void wipe(void *p, std::size_t n) {
  volatile std::uint8_t *v = static_cast<volatile std::uint8_t *>(p);
  for (std::size_t i = 0; i < n; ++i) v[i] = 0;
}

[[noreturn]] void throw_status(int rc) {
  if (rc == NOISE_GPU_E_MAC) throw std::invalid_argument("Invalid MAC");
  if (rc == NOISE_GPU_E_NONCE) throw std::out_of_range("Nonce limit has been exceeded!");
  if (rc == NOISE_GPU_E_ARG) throw std::invalid_argument(noise_gpu_last_error());
  throw std::runtime_error(std::string("noise-mi355x: ") + noise_gpu_strerror(rc) +
                           ": " + noise_gpu_last_error());
}

// How many of `count` sequential records starting at nonce n may be
// processed before reaching the limit (noise.cpp:398: n == 2^64-2 throws).
std::uint64_t records_before_limit(std::uint64_t n, std::uint64_t count) {
  const std::uint64_t room = kNonceLimit - n;  // mod 2^64; 2^64-1 when n == UINT64_MAX
  return std::min(count, room);
}

}  // namespace

void encrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out) {
  const std::size_t text_size = in_out.size();
  in_out.resize(text_size + 16);
  const int rc = noise_gpu_encrypt_host(k.data(), n, ad ? ad->data() : nullptr, ad ? ad->size() : 0,
                                        in_out.data(), text_size);
  wipe(k.data(), k.size());  // noise.cpp:222
  if (rc != NOISE_GPU_OK) {
    in_out.resize(text_size);
    throw_status(rc);
  }
}

void decrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out) {
  const int rc = in_out.size() < 16
                     ? NOISE_GPU_E_MAC
                     : noise_gpu_decrypt_host(k.data(), n, ad ? ad->data() : nullptr, ad ? ad->size() : 0,
                                              in_out.data(), in_out.size());
  wipe(k.data(), k.size());  // noise.cpp:272-273 / 278
  if (rc != NOISE_GPU_OK) throw_status(rc);
  in_out.resize(in_out.size() - 16);
}

CipherState::~CipherState() {
  wipe(k.data(), k.size());
  n = std::numeric_limits<std::uint64_t>::max();
}

void CipherState::initialize_key(const std::array<std::uint8_t, 32> &key) {
  k = key;
  n = 0;
}

bool CipherState::has_key() const {
  std::uint8_t acc = 0;
  for (auto b : k) acc |= b;
  return acc != 0;
}

void CipherState::set_nonce(const std::uint64_t &nonce) { n = nonce; }

void CipherState::encrypt_raw(const std::uint8_t *ad, std::size_t ad_len,
                              std::vector<std::uint8_t> &plaintext) {
  if (n == kNonceLimit) throw std::out_of_range("Nonce limit has been exceeded!");
  const std::size_t len = plaintext.size();
  plaintext.resize(len + 16);
  const int rc = noise_gpu_encrypt_host(k.data(), n, ad, ad_len, plaintext.data(), len);
  if (rc != NOISE_GPU_OK) {
    plaintext.resize(len);
    throw_status(rc);
  }
  ++n;
}

void CipherState::decrypt_raw(const std::uint8_t *ad, std::size_t ad_len,
                              std::vector<std::uint8_t> &ciphertext) {
  if (n == kNonceLimit) throw std::out_of_range("Nonce limit has been exceeded!");
  const std::uint64_t nonce = n++;  // advances even on MAC failure (noise.cpp:421)
  const int rc = noise_gpu_decrypt_host(k.data(), nonce, ad, ad_len,
                                        ciphertext.data(), ciphertext.size());
  if (rc != NOISE_GPU_OK) throw_status(rc);
  ciphertext.resize(ciphertext.size() - 16);
}

void CipherState::encrypt_with_ad(std::vector<std::uint8_t> &plaintext) {
  std::vector<std::uint8_t> null_ad;
  encrypt_with_ad(null_ad, plaintext);
}

void CipherState::decrypt_with_ad(std::vector<std::uint8_t> &ciphertext) {
  std::vector<std::uint8_t> null_ad;
  decrypt_with_ad(null_ad, ciphertext);
}

void CipherState::rekey() {
  // k <- ENCRYPT(k, 2^64-2, empty, 0^32)[0..32) -- no has_key gate, as in
  // the reference (noise.cpp:429-439).
  std::array<std::uint8_t, 32> tmp = k;
  const int rc = noise_gpu_rekey_host(tmp.data());
  if (rc != NOISE_GPU_OK) {
    wipe(tmp.data(), tmp.size());
    throw_status(rc);
  }
  k = tmp;
  wipe(tmp.data(), tmp.size());
}

void CipherState::encrypt_batch(std::vector<std::vector<std::uint8_t>> &messages) {
  if (!has_key() || messages.empty()) return;
  const std::uint64_t todo = records_before_limit(n, messages.size());
  // One descriptor-kernel launch over all messages (16-byte aligned slots
  // so uniform-length traffic takes the dwordx4 path).
  std::vector<noise_gpu_record> recs(todo);
  std::uint64_t in_bytes = 0, out_bytes = 0;
  for (std::uint64_t i = 0; i < todo; ++i) {
    const std::uint32_t len = (std::uint32_t)messages[i].size();
    recs[i] = noise_gpu_record{in_bytes, out_bytes, n + i, 0, len, 0, 0, 0};
    in_bytes += (len + 15) & ~15u;
    out_bytes += (len + 16 + 15) & ~15u;
  }
  if (todo) {
    std::vector<std::uint8_t> hin(in_bytes), hout(out_bytes);
    for (std::uint64_t i = 0; i < todo; ++i)
      std::memcpy(hin.data() + recs[i].in_off, messages[i].data(), messages[i].size());
    const int rc = noise_gpu_encrypt_records_host(k.data(), 1, recs.data(), todo,
                                                  hin.data(), in_bytes, hout.data(),
                                                  out_bytes, nullptr, 0);
    wipe(hin.data(), hin.size());
    if (rc != NOISE_GPU_OK) throw_status(rc);
    for (std::uint64_t i = 0; i < todo; ++i) {
      auto &m = messages[i];
      m.resize(m.size() + 16);
      std::memcpy(m.data(), hout.data() + recs[i].out_off, m.size());
    }
    n += todo;
  }
  if (todo < messages.size()) throw std::out_of_range("Nonce limit has been exceeded!");
}

void CipherState::decrypt_batch(std::vector<std::vector<std::uint8_t>> &messages,
                                std::vector<std::uint8_t> *ok) {
  if (ok) ok->assign(messages.size(), 0);
  if (!has_key() || messages.empty()) return;
  const std::uint64_t todo = records_before_limit(n, messages.size());
  std::vector<noise_gpu_record> recs(todo);
  std::vector<std::uint8_t> short_rec(todo, 0);
  std::uint64_t in_bytes = 0, out_bytes = 0;
  for (std::uint64_t i = 0; i < todo; ++i) {
    const std::size_t sz = messages[i].size();
    const std::uint32_t len = sz >= 16 ? (std::uint32_t)(sz - 16) : 0;
    short_rec[i] = sz < 16;
    recs[i] = noise_gpu_record{in_bytes, out_bytes, n + i, 0, len, 0, 0, 0};
    in_bytes += (len + 16 + 15) & ~15u;
    out_bytes += (len + 15) & ~15u;
  }
  bool any_bad = false;
  if (todo) {
    std::vector<std::uint8_t> hin(in_bytes), hout(out_bytes), st(todo, 1);
    for (std::uint64_t i = 0; i < todo; ++i)
      if (!short_rec[i])
        std::memcpy(hin.data() + recs[i].in_off, messages[i].data(), messages[i].size());
    const int rc = noise_gpu_decrypt_records_host(k.data(), 1, recs.data(), todo,
                                                  hin.data(), in_bytes, hout.data(),
                                                  out_bytes, nullptr, 0, st.data());
    if (rc != NOISE_GPU_OK) throw_status(rc);
    for (std::uint64_t i = 0; i < todo; ++i) {
      const bool good = !short_rec[i] && st[i] == NOISE_GPU_REC_OK;
      if (ok) (*ok)[i] = good;
      if (!good) { any_bad = true; continue; }
      auto &m = messages[i];
      m.resize(m.size() - 16);
      std::memcpy(m.data(), hout.data() + recs[i].out_off, m.size());
    }
    wipe(hout.data(), hout.size());
    n += todo;  // every attempted record consumes its nonce (noise.cpp:421)
  }
  if (todo < messages.size()) throw std::out_of_range("Nonce limit has been exceeded!");
  if (any_bad) throw std::invalid_argument("Invalid MAC");
}

void CipherState::encrypt_device(const std::uint8_t *d_in, std::uint64_t in_stride,
                                 std::uint8_t *d_out, std::uint64_t out_stride,
                                 std::uint32_t len, std::uint64_t count, void *stream) {
  if (!has_key() || count == 0) return;
  const std::uint64_t todo = records_before_limit(n, count);
  if (todo) {
    const int rc = noise_gpu_encrypt_uniform(k.data(), n, d_in, in_stride, d_out,
                                             out_stride, len, nullptr, 0, 0, todo, stream);
    if (rc != NOISE_GPU_OK) throw_status(rc);
    n += todo;
  }
  if (todo < count) throw std::out_of_range("Nonce limit has been exceeded!");
}

void CipherState::decrypt_device(const std::uint8_t *d_in, std::uint64_t in_stride,
                                 std::uint8_t *d_out, std::uint64_t out_stride,
                                 std::uint32_t len, std::uint8_t *d_status,
                                 std::uint64_t count, void *stream) {
  if (!has_key() || count == 0) return;
  const std::uint64_t todo = records_before_limit(n, count);
  if (todo) {
    const int rc = noise_gpu_decrypt_uniform(k.data(), n, d_in, in_stride, d_out,
                                             out_stride, len, nullptr, 0, 0, d_status,
                                             todo, stream);
    if (rc != NOISE_GPU_OK) throw_status(rc);
    n += todo;
  }
  if (todo < count) throw std::out_of_range("Nonce limit has been exceeded!");
}

}  // namespace noise
