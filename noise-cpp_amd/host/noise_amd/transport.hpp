// noise_amd/transport.hpp -- the data formats either side of the AEAD path
// (SURVEY.md §8(f) rank 2): Noise messages on a byte stream and many
// sessions' records batched into one device launch.
//
// The reference leaves transport to the caller (README.md:31-54): a message
// is at most 65535 bytes (noise.cpp:886, 982), and the Noise spec (rev34 §3)
// frames stream transports with a 2-byte big-endian length.  Here:
//   * append_frame / Deframer: that framing, incremental over arbitrary
//     socket-read chunks;
//   * Batcher: queued messages of many sessions (each a CipherState: key +
//     next nonce) -> ONE descriptor batch on the GPU (noise_gpu_encrypt_
//     records_host / _decrypt_records_host) -> per-message results in
//     submission order.  Nonces are assigned at submit in each session's
//     order, exactly as consecutive encrypt_with_ad / decrypt_with_ad calls
//     would (decrypt advances n even when the tag fails, noise.cpp:421; the
//     nonce limit 2^64-2 throws out_of_range, noise.cpp:398-400).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "noise_amd/cipher_state.hpp"

namespace noise::transport {

constexpr std::size_t kMaxMessage = 65535;

// stream || BE16(len) || msg; throws length_error if len > 65535
void append_frame(std::vector<std::uint8_t> &stream, const std::uint8_t *msg, std::size_t len);

// Incremental parser of BE16-length-prefixed messages.
class Deframer {
 public:
  void feed(const std::uint8_t *p, std::size_t n);
  // next complete message (false if none buffered yet)
  bool next(std::vector<std::uint8_t> &msg);
  [[nodiscard]] std::size_t buffered() const { return buf_.size() - pos_; }

 private:
  std::vector<std::uint8_t> buf_;
  std::size_t pos_ = 0;
};

class Batcher {
 public:
  enum class Direction { Encrypt, Decrypt };
  struct Result {
    std::size_t session;
    std::uint64_t nonce;
    bool ok;                         // decrypt: tag verified
    std::vector<std::uint8_t> msg;   // ct || tag (encrypt) / plaintext (decrypt, if ok)
  };

  explicit Batcher(Direction d) : dir_(d) {}
  // register a session: its key and next nonce (copied); returns its id
  std::size_t add_session(const CipherState &cs);
  // queue one message of session s (plaintext / ct || tag)
  void submit(std::size_t s, std::vector<std::uint8_t> msg);
  [[nodiscard]] std::size_t pending() const { return queue_.size(); }
  // every queued message in one GPU launch; results in submission order
  std::vector<Result> flush();
  [[nodiscard]] std::uint64_t nonce(std::size_t s) const { return sessions_.at(s).n; }
  // a CipherState that continues session s (same key, next nonce)
  [[nodiscard]] CipherState state(std::size_t s) const;

 private:
  struct Session {
    std::array<std::uint8_t, 32> k;
    std::uint64_t n;
  };
  struct Item {
    std::size_t session;
    std::uint64_t nonce;
    std::vector<std::uint8_t> msg;
  };
  Direction dir_;
  std::vector<Session> sessions_;
  std::vector<Item> queue_;
};

}  // namespace noise::transport
