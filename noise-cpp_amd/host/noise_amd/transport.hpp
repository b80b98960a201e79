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
//     nonce limit 2^64-2 throws out_of_range, noise.cpp:398-400);
//   * Pipeline: the same batching over pinned ring slots for serving: a
//     message is copied ONCE, from the caller's socket buffer into the
//     pinned slot being filled; flush() launches that slot asynchronously
//     (H2D, the records kernels, D2H on the slot's own stream) and filling
//     continues in the next slot, so host copies, PCIe and the GPU overlap.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
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
  // register a session: its key and next nonce (copied); returns its id.
  // Throws invalid_argument for a CipherState without a key (has_key()
  // false): the GPU never uses an all-zero key row.
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

// Pinned, multi-slot, asynchronous form of Batcher (same nonce / length /
// failure semantics).  Usage:
//   Pipeline p(Pipeline::Direction::Encrypt);
//   auto s = p.add_session(cs);
//   while (more) { if (!p.submit(s, buf, n)) { tickets.push(p.flush()); p.submit(s, buf, n); } }
//   auto b = p.wait(tickets.front());   // b.data(i) / b.length(i) / b.ok(i)
// A Batch view stays valid until its slot is refilled, i.e. until `depth - 1`
// further flushes; flush() blocks only when the slot it moves on to is still
// in flight (back-pressure).  With Options::launch_thread the slot's HIP work
// is enqueued by a launcher thread, so flush() returns at once and the
// enqueue overlaps the caller's copies; an enqueue error is rethrown by the
// next flush() / wait().  The launcher uses the device current when the
// Pipeline was built.  Session keys are uploaded to a device key table
// once, when the session is added.  One thread drives a Pipeline (like
// CipherState); submit_batch / copy_out fan the byte copies out to an
// internal pool of Options::copy_threads threads.
class Pipeline {
 public:
  using Direction = Batcher::Direction;
  struct Options {
    std::size_t slot_bytes = std::size_t(32) << 20;  // message bytes per slot
    std::size_t slot_records = std::size_t(1) << 17; // messages per slot (48-B descriptors)
    int depth = 4;  // slots in the ring: one filling, depth - 2 in flight while
                    // the oldest is consumed (a slot's copies take ~1.3 ms at 32 MiB)
    int copy_threads = 1;  // host threads copying messages in / results out
                           // (submit_batch, copy_out); 1 = the caller only
    bool launch_thread = true;  // flush() hands a slot's HIP enqueue (copies,
                                // kernels, event) to a thread of its own
  };
  struct Message {
    std::size_t session;
    const std::uint8_t *data;
    std::size_t len;
  };
  class Batch {
   public:
    [[nodiscard]] std::size_t size() const { return n_; }
    [[nodiscard]] std::size_t session(std::size_t i) const;
    [[nodiscard]] std::uint64_t nonce(std::size_t i) const;
    [[nodiscard]] bool ok(std::size_t i) const;                 // decrypt: tag verified
    [[nodiscard]] const std::uint8_t *data(std::size_t i) const;  // ct || tag / plaintext
    [[nodiscard]] std::size_t length(std::size_t i) const;

   private:
    friend class Pipeline;
    const std::uint8_t *h_ = nullptr;
    std::size_t n_ = 0, o_out_ = 0, o_st_ = 0;
    bool dec_ = false;
  };

  explicit Pipeline(Direction d) : Pipeline(d, Options{}) {}
  Pipeline(Direction d, const Options &o);
  ~Pipeline();
  Pipeline(const Pipeline &) = delete;
  Pipeline &operator=(const Pipeline &) = delete;

  // as Batcher::add_session (a keyless CipherState throws invalid_argument)
  std::size_t add_session(const CipherState &cs);
  // copy one message into the filling slot and assign its nonce; false (and
  // nothing consumed) when the slot has no room -- flush() and retry
  bool submit(std::size_t s, const std::uint8_t *msg, std::size_t len);
  // Queue the longest prefix of messages[0..n) that fits the filling slot,
  // exactly as that many submit() calls would (nonces in order per session,
  // the same length / nonce-limit exceptions), with the byte copies spread
  // over Options::copy_threads threads.  Returns how many were queued; 0
  // means the slot is full: flush() and call again.
  std::size_t submit_batch(const Message *messages, std::size_t n);
  // copy a waited batch's results out (dst[i] <- data(i), length(i) bytes),
  // over Options::copy_threads threads
  void copy_out(const Batch &b, std::uint8_t *const *dst);
  [[nodiscard]] std::size_t pending() const;
  // launch the filling slot; its ticket (0 if it was empty)
  std::uint64_t flush();
  // block until a flushed slot is done
  Batch wait(std::uint64_t ticket);
  [[nodiscard]] std::uint64_t nonce(std::size_t s) const { return nonces_.at(s); }
  [[nodiscard]] CipherState state(std::size_t s) const;

 private:
  struct Slot;
  void sync_all();
  void grow_keys();
  struct LaunchJob;
  void enqueue(const LaunchJob &j);  // the slot's HIP work, in stream order
  void wait_enqueued(Slot &sl);      // the launcher has issued sl's work
  struct Launcher;
  std::unique_ptr<Launcher> launcher_;
  int dev_ = 0;
  Direction dir_;
  Options opt_;
  std::size_t o_in_ = 0, o_out_ = 0, o_st_ = 0, slot_total_ = 0;
  std::vector<Slot *> slots_;
  std::size_t fill_ = 0;          // slot being filled
  std::uint64_t tickets_ = 0;
  std::vector<std::uint64_t> nonces_;
  std::uint8_t *h_keys_ = nullptr, *d_keys_ = nullptr;  // pinned mirror / device table
  std::size_t key_cap_ = 0, key_dirty_ = 0;
  std::vector<std::uint8_t *> retired_h_;  // outgrown pinned key mirrors (wiped)
  void *keys_evt_ = nullptr;  // hipEvent_t: latest key-row upload (any slot stream)
  bool keys_uploaded_ = false;
  struct CopyPool;
  std::unique_ptr<CopyPool> pool_;
  // submit_batch's parallel bookkeeping: per copy thread, its messages' count
  // per session and byte totals (scratch kept across calls)
  std::vector<std::uint32_t> sess_cnt_;
  std::size_t submit_serial(const Message *messages, std::size_t n);
};

}  // namespace noise::transport
