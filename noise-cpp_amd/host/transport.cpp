// transport.cpp -- stream framing and the multi-session batcher over the
// descriptor-batch C ABI (noise_amd/transport.hpp).
#include "noise_amd/transport.hpp"

#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include <hip/hip_runtime_api.h>

#include "noise_amd/dev_mem.hpp"
#include "noise_gpu.h"

namespace noise::transport {

using noise_amd::dev_alloc;
using noise_amd::dev_wipe_free;

void append_frame(std::vector<std::uint8_t> &stream, const std::uint8_t *msg, std::size_t len) {
  if (len > kMaxMessage) throw std::length_error("Noise message exceeds 65535 bytes");
  stream.push_back((std::uint8_t)(len >> 8));
  stream.push_back((std::uint8_t)len);
  stream.insert(stream.end(), msg, msg + len);
}

void Deframer::feed(const std::uint8_t *p, std::size_t n) {
  if (pos_ > 0 && pos_ == buf_.size()) {
    buf_.clear();
    pos_ = 0;
  } else if (pos_ > (1u << 20)) {  // compact consumed bytes now and then
    buf_.erase(buf_.begin(), buf_.begin() + (std::ptrdiff_t)pos_);
    pos_ = 0;
  }
  buf_.insert(buf_.end(), p, p + n);
}

bool Deframer::next(std::vector<std::uint8_t> &msg) {
  if (buf_.size() - pos_ < 2) return false;
  const std::size_t len = ((std::size_t)buf_[pos_] << 8) | buf_[pos_ + 1];
  if (buf_.size() - pos_ - 2 < len) return false;
  msg.assign(buf_.begin() + (std::ptrdiff_t)(pos_ + 2), buf_.begin() + (std::ptrdiff_t)(pos_ + 2 + len));
  pos_ += 2 + len;
  return true;
}

// A session without a key (HasKey() false: an all-zero key) is refused.  The
// batch kernels never use an all-zero key row (they write nothing and report
// NOISE_GPU_REC_BAD_KEY), so such a session's results would be garbage
// reported as valid ciphertext; the reference CipherState would instead pass
// the plaintext through unencrypted (noise.cpp:395-397), which a batch API
// must not do silently either.
static void require_key(const CipherState &cs) {
  if (!cs.has_key()) throw std::invalid_argument("transport: session has no key");
}

std::size_t Batcher::add_session(const CipherState &cs) {
  require_key(cs);
  sessions_.push_back({cs.key_material(), cs.nonce()});
  return sessions_.size() - 1;
}

CipherState Batcher::state(std::size_t s) const {
  const Session &ss = sessions_.at(s);
  CipherState cs;
  cs.initialize_key(ss.k);
  cs.set_nonce(ss.n);
  return cs;
}

void Batcher::submit(std::size_t s, std::vector<std::uint8_t> msg) {
  Session &ss = sessions_.at(s);
  if (ss.n == std::numeric_limits<std::uint64_t>::max() - 1)  // noise.cpp:398-400
    throw std::out_of_range("Nonce limit has been exceeded!");
  if (dir_ == Direction::Encrypt && msg.size() + 16 > kMaxMessage)
    throw std::length_error("Noise message exceeds 65535 bytes");
  if (dir_ == Direction::Decrypt && (msg.size() < 16 || msg.size() > kMaxMessage))
    throw std::invalid_argument("Invalid MAC");  // shorter than a tag
  queue_.push_back({s, ss.n, std::move(msg)});
  ++ss.n;  // decrypt: advances whatever the tag says (noise.cpp:421)
}

std::vector<Batcher::Result> Batcher::flush() {
  std::vector<Result> out;
  if (queue_.empty()) return out;
  const bool dec = dir_ == Direction::Decrypt;
  const std::size_t nrec = queue_.size();
  std::vector<noise_gpu_record> recs(nrec);
  std::uint64_t in_bytes = 0, out_bytes = 0;
  for (std::size_t i = 0; i < nrec; ++i) {  // 16-byte aligned slots: the tile kernels' layout
    const std::uint64_t len = dec ? queue_[i].msg.size() - 16 : queue_[i].msg.size();
    const std::uint64_t in_len = dec ? len + 16 : len, out_len = dec ? len : len + 16;
    recs[i] = noise_gpu_record{in_bytes, out_bytes, queue_[i].nonce, 0, (std::uint32_t)len, 0,
                               (std::uint32_t)queue_[i].session, 0};
    in_bytes += (in_len + 15) / 16 * 16;
    out_bytes += (out_len + 15) / 16 * 16;
  }
  std::vector<std::uint8_t> in(in_bytes ? in_bytes : 1), outb(out_bytes ? out_bytes : 1), st(nrec);
  for (std::size_t i = 0; i < nrec; ++i)
    if (!queue_[i].msg.empty()) std::memcpy(in.data() + recs[i].in_off, queue_[i].msg.data(), queue_[i].msg.size());
  std::vector<std::uint8_t> keys(32 * sessions_.size());
  for (std::size_t s = 0; s < sessions_.size(); ++s) std::memcpy(keys.data() + 32 * s, sessions_[s].k.data(), 32);
  const int rc = dec ? noise_gpu_decrypt_records_host(keys.data(), (std::uint32_t)sessions_.size(), recs.data(),
                                                      nrec, in.data(), in_bytes, outb.data(), out_bytes,
                                                      nullptr, 0, st.data())
                     : noise_gpu_encrypt_records_host(keys.data(), (std::uint32_t)sessions_.size(), recs.data(),
                                                      nrec, in.data(), in_bytes, outb.data(), out_bytes,
                                                      nullptr, 0);
  volatile std::uint8_t *kv = keys.data();
  for (std::size_t i = 0; i < keys.size(); ++i) kv[i] = 0;
  if (rc != NOISE_GPU_OK)
    throw std::runtime_error(std::string("noise-mi355x: ") + noise_gpu_strerror(rc) + ": " +
                             noise_gpu_last_error());
  out.reserve(nrec);
  for (std::size_t i = 0; i < nrec; ++i) {
    Result r{queue_[i].session, queue_[i].nonce, !dec || st[i] == NOISE_GPU_REC_OK, {}};
    const std::size_t olen = dec ? recs[i].len : recs[i].len + 16;
    if (r.ok) r.msg.assign(outb.begin() + (std::ptrdiff_t)recs[i].out_off,
                           outb.begin() + (std::ptrdiff_t)(recs[i].out_off + olen));
    out.push_back(std::move(r));
  }
  queue_.clear();
  return out;
}

// ---- Pipeline ---------------------------------------------------------------
namespace {
void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("noise-mi355x pipeline: ") + what + ": " + hipGetErrorString(e));
}
inline std::size_t align16(std::size_t x) { return (x + 15) & ~std::size_t(15); }
inline std::size_t align256(std::size_t x) { return (x + 255) & ~std::size_t(255); }

// Bulk message copy with streaming (non-temporal) stores.  A plain memcpy of
// a 1 KiB message into a cold destination line first reads the line for
// ownership, so every copied byte costs three memory transfers; streaming
// stores write whole lines and skip that read.  The destination must be
// 16-byte aligned (slot offsets are; so are the caller's result buffers in
// the common case -- otherwise plain memcpy).  The caller issues
// stream_fence() before anyone else (a DMA engine, another thread) reads.
typedef std::uint32_t v4u32 __attribute__((ext_vector_type(4)));
inline void stream_copy(std::uint8_t *dst, const std::uint8_t *src, std::size_t n) {
  if (n < 256 || (reinterpret_cast<std::uintptr_t>(dst) & 15u) != 0) {
    std::memcpy(dst, src, n);
    return;
  }
  std::size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    v4u32 a, b, c, d;
    std::memcpy(&a, src + i, 16);
    std::memcpy(&b, src + i + 16, 16);
    std::memcpy(&c, src + i + 32, 16);
    std::memcpy(&d, src + i + 48, 16);
    __builtin_nontemporal_store(a, reinterpret_cast<v4u32 *>(dst + i));
    __builtin_nontemporal_store(b, reinterpret_cast<v4u32 *>(dst + i + 16));
    __builtin_nontemporal_store(c, reinterpret_cast<v4u32 *>(dst + i + 32));
    __builtin_nontemporal_store(d, reinterpret_cast<v4u32 *>(dst + i + 48));
  }
  if (i < n) std::memcpy(dst + i, src + i, n - i);
}
inline void stream_fence() { __builtin_ia32_sfence(); }
}  // namespace

// Fork-join pool for the host byte copies (submit_batch / copy_out): the
// caller runs chunk 0 of every job, workers 1..T-1 the others.
struct Pipeline::CopyPool {
  explicit CopyPool(int threads) : nthr(threads < 1 ? 1 : threads) {
    for (int w = 1; w < nthr; ++w) th.emplace_back([this, w] { worker(w); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  // fn(lo, hi) over [0, n) in nthr contiguous chunks
  void run(std::size_t n, const std::function<void(std::size_t, std::size_t)> &fn) {
    run_idx(n, [&fn](std::size_t, std::size_t lo, std::size_t hi) { fn(lo, hi); });
  }
  // fn(c, lo, hi): chunk c of [0, n) is [n c / nthr, n (c + 1) / nthr) --
  // or, below 64 items or with one thread, chunk 0 is all of [0, n) and the
  // others do not run.  The caller is given c, so a chunk's index never has
  // to be re-derived from lo (empty chunks when n < nthr share their lo).
  void run_idx(std::size_t n, const std::function<void(std::size_t, std::size_t, std::size_t)> &fn) {
    if (nthr == 1 || n < 64) {
      fn(0, 0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      job = &fn;
      total = n;
      pending = nthr - 1;
      ++gen;
    }
    cv.notify_all();
    fn(0, 0, n / nthr);
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [this] { return pending == 0; });
    job = nullptr;
  }
  void worker(int w) {
    std::uint64_t seen = 0;
    for (;;) {
      const std::function<void(std::size_t, std::size_t, std::size_t)> *fn;
      std::size_t n;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        fn = job;
        n = total;
      }
      (*fn)((std::size_t)w, n * w / nthr, n * (w + 1) / nthr);
      {
        std::lock_guard<std::mutex> lk(mu);
        if (--pending == 0) done.notify_one();
      }
    }
  }
  int nthr;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done;
  const std::function<void(std::size_t, std::size_t, std::size_t)> *job = nullptr;
  std::size_t total = 0;
  std::uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
};

// One ring slot: pinned host image and device image of
// [records | message bytes in | message bytes out | status]
struct Pipeline::Slot {
  std::uint8_t *h = nullptr, *d = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  std::size_t nrec = 0, in_used = 0, out_used = 0;
  std::uint64_t ticket = 0;
  bool in_flight = false;
  bool enqueued = true;  // the launcher has issued its work (Launcher::mu)
  noise_gpu_record *recs() { return reinterpret_cast<noise_gpu_record *>(h); }
};

// What flush() hands over: the slot and the key rows it needs uploaded,
// snapshotted on the caller's thread (add_session() may append rows after).
struct Pipeline::LaunchJob {
  Slot *sl;
  std::size_t key_lo, nkeys;
};

// The launcher thread.  A flush costs ~15 HIP calls (~0.15-0.4 ms of API
// time at 32 MiB slots: H2D, the records call's kernels, D2H, the event);
// on the caller's thread that time sat between the byte copies of
// consecutive slots.  Jobs run in flush order, so stream order and the key
// upload order are the caller's.
struct Pipeline::Launcher {
  std::mutex mu;
  std::condition_variable cv, issued;
  std::deque<LaunchJob> q;
  bool stop = false;
  std::exception_ptr err;  // first enqueue failure; the Pipeline is unusable after it
  std::thread th;
};

Pipeline::Pipeline(Direction d, const Options &o) : dir_(d), opt_(o) {
  hip_check(hipGetDevice(&dev_), "current device");
  if (opt_.depth < 2 || opt_.slot_records == 0 || opt_.slot_bytes < 65536)
    throw std::invalid_argument("pipeline: depth >= 2, slot_records >= 1, slot_bytes >= 64 KiB");
  o_in_ = align256(opt_.slot_records * sizeof(noise_gpu_record));
  o_out_ = align256(o_in_ + opt_.slot_bytes);
  o_st_ = align256(o_out_ + opt_.slot_bytes + 16 * opt_.slot_records);
  slot_total_ = o_st_ + opt_.slot_records;
  for (int i = 0; i < opt_.depth; ++i) {
    Slot *sl = new Slot();
    slots_.push_back(sl);
    hip_check(hipHostMalloc(reinterpret_cast<void **>(&sl->h), slot_total_, hipHostMallocDefault),
              "pinned slot");
    hip_check(hipStreamCreateWithFlags(&sl->st, hipStreamNonBlocking), "slot stream");
    hip_check(dev_alloc(reinterpret_cast<void **>(&sl->d), slot_total_, sl->st), "device slot");
    hip_check(hipStreamSynchronize(sl->st), "device slot");
    hip_check(hipEventCreateWithFlags(&sl->done, hipEventDisableTiming), "slot event");
  }
  pool_ = std::make_unique<CopyPool>(opt_.copy_threads);
  hipEvent_t ke = nullptr;
  hip_check(hipEventCreateWithFlags(&ke, hipEventDisableTiming), "key event");
  keys_evt_ = ke;
  if (opt_.launch_thread) {
    launcher_ = std::make_unique<Launcher>();
    Launcher *L = launcher_.get();
    L->th = std::thread([this, L] {
      const hipError_t de = hipSetDevice(dev_);
      std::unique_lock<std::mutex> lk(L->mu);
      for (;;) {
        L->cv.wait(lk, [L] { return L->stop || !L->q.empty(); });
        if (L->q.empty()) return;  // stop, queue drained
        const LaunchJob j = L->q.front();
        L->q.pop_front();
        lk.unlock();
        std::exception_ptr e;
        try {
          if (!L->err) {  // after a failure nothing more is issued
            hip_check(de, "launcher device");
            enqueue(j);
          }
        } catch (...) {
          e = std::current_exception();
        }
        lk.lock();
        if (e && !L->err) L->err = e;
        j.sl->enqueued = true;
        L->issued.notify_all();
      }
    });
  }
}

void Pipeline::wait_enqueued(Slot &sl) {
  if (!launcher_) return;
  Launcher &L = *launcher_;
  std::unique_lock<std::mutex> lk(L.mu);
  L.issued.wait(lk, [&] { return sl.enqueued; });
  if (L.err) std::rethrow_exception(L.err);
}

Pipeline::~Pipeline() {
  if (launcher_) {  // issue what was flushed, then stop
    {
      std::lock_guard<std::mutex> lk(launcher_->mu);
      launcher_->stop = true;
    }
    launcher_->cv.notify_all();
    launcher_->th.join();
    launcher_->err = nullptr;  // sync_all below waits for whatever was issued
  }
  try {
    sync_all();
  } catch (...) {
  }
  if (h_keys_) {
    volatile std::uint8_t *kv = h_keys_;
    for (std::size_t i = 0; i < 32 * key_cap_; ++i) kv[i] = 0;
    (void)hipHostFree(h_keys_);
  }
  for (std::uint8_t *p : retired_h_) (void)hipHostFree(p);  // wiped when retired
  // Device memory is wiped and freed stream-ordered on the slot streams
  // (dev_mem.hpp), after sync_all: no device-wide wait, so a resident latency
  // instance serving another thread does not hold this up.  (hipHostFree
  // below still waits for every stream of the device: noise_gpu.h.)
  // Everything below on the Pipeline's device (the frees, their
  // pool choice and the records scratch release all follow the current device)
  const noise_amd::DeviceGuard on_dev(dev_);
  if (d_keys_) {
    (void)dev_wipe_free(d_keys_, 32 * key_cap_, slots_[0]->st);
    (void)hipStreamSynchronize(slots_[0]->st);
  }
  // the records scratch and companion stream cached for each slot stream go
  // with it
  for (Slot *sl : slots_)
    if (sl->st) (void)noise_gpu_scratch_release(sl->st);
  for (Slot *sl : slots_) {
    if (sl->d && sl->st) {  // the messages in and out: wiped, then freed
      (void)dev_wipe_free(sl->d, slot_total_, sl->st);
      (void)hipStreamSynchronize(sl->st);
    }
    if (sl->h) {
      std::memset(sl->h, 0, slot_total_);
      (void)hipHostFree(sl->h);
    }
    if (sl->st) (void)hipStreamDestroy(sl->st);
    if (sl->done) (void)hipEventDestroy(sl->done);
    delete sl;
  }
  if (keys_evt_) (void)hipEventDestroy(static_cast<hipEvent_t>(keys_evt_));
}

void Pipeline::sync_all() {
  for (Slot *sl : slots_)
    if (sl->in_flight) {
      wait_enqueued(*sl);
      hip_check(hipEventSynchronize(sl->done), "slot wait");
    }
}

void Pipeline::grow_keys() {
  // the device table may be read by slots in flight: let them finish first
  // (sync_all also waits until the launcher has issued every flushed slot, so
  // nothing else enqueues on slot 0's stream, which carries the table below)
  sync_all();
  const noise_amd::DeviceGuard on_dev(dev_);  // the table lives on the Pipeline's device
  const std::size_t cap = key_cap_ ? 2 * key_cap_ : 1024;
  hipStream_t ks = slots_[0]->st;
  std::uint8_t *h = nullptr, *d = nullptr;
  hip_check(hipHostMalloc(reinterpret_cast<void **>(&h), 32 * cap, hipHostMallocDefault), "pinned keys");
  // stream-ordered (dev_mem.hpp): no device-wide wait here, so a resident
  // latency instance on another thread cannot hold up add_session()
  hip_check(dev_alloc(reinterpret_cast<void **>(&d), 32 * cap, ks), "device keys");
  if (key_cap_) {
    std::memcpy(h, h_keys_, 32 * key_cap_);
    hip_check(hipMemcpyAsync(d, d_keys_, 32 * key_cap_, hipMemcpyDeviceToDevice, ks), "key table copy");
    hip_check(dev_wipe_free(d_keys_, 32 * key_cap_, ks), "old key table");
  }
  hip_check(hipStreamSynchronize(ks), "key table");
  if (key_cap_) {
    // the old pinned mirror is wiped now and freed with the Pipeline:
    // hipHostFree waits for every stream of the device (noise_gpu.h), and
    // the mirrors double, so the retired ones add up to less than the current
    volatile std::uint8_t *kv = h_keys_;
    for (std::size_t i = 0; i < 32 * key_cap_; ++i) kv[i] = 0;
    retired_h_.push_back(h_keys_);
  }
  h_keys_ = h;
  d_keys_ = d;
  key_cap_ = cap;
}

std::size_t Pipeline::add_session(const CipherState &cs) {
  require_key(cs);
  const std::size_t s = nonces_.size();
  if (s >= 0xffffffffu) throw std::length_error("pipeline: too many sessions");
  if (s == key_cap_) grow_keys();
  const std::array<std::uint8_t, 32> k = cs.key_material();
  std::memcpy(h_keys_ + 32 * s, k.data(), 32);
  nonces_.push_back(cs.nonce());
  return s;
}

CipherState Pipeline::state(std::size_t s) const {
  if (s >= nonces_.size()) throw std::out_of_range("pipeline: no such session");
  std::array<std::uint8_t, 32> k;
  std::memcpy(k.data(), h_keys_ + 32 * s, 32);
  CipherState cs;
  cs.initialize_key(k);
  cs.set_nonce(nonces_[s]);
  return cs;
}

std::size_t Pipeline::pending() const { return slots_[fill_]->nrec; }

bool Pipeline::submit(std::size_t s, const std::uint8_t *msg, std::size_t len) {
  std::uint64_t &n = nonces_.at(s);
  const bool dec = dir_ == Direction::Decrypt;
  if (n == std::numeric_limits<std::uint64_t>::max() - 1)  // noise.cpp:398-400
    throw std::out_of_range("Nonce limit has been exceeded!");
  if (!dec && len + 16 > kMaxMessage) throw std::length_error("Noise message exceeds 65535 bytes");
  if (dec && (len < 16 || len > kMaxMessage)) throw std::invalid_argument("Invalid MAC");
  Slot &sl = *slots_[fill_];
  const std::size_t in_len = align16(len), out_len = dec ? align16(len - 16) : align16(len + 16);
  if (sl.nrec == opt_.slot_records || sl.in_used + in_len > opt_.slot_bytes) return false;
  if (len) std::memcpy(sl.h + o_in_ + sl.in_used, msg, len);
  sl.recs()[sl.nrec] = noise_gpu_record{sl.in_used, sl.out_used, n, 0,
                                        (std::uint32_t)(dec ? len - 16 : len), 0,
                                        (std::uint32_t)s, 0};
  sl.in_used += in_len;
  sl.out_used += out_len;
  ++sl.nrec;
  ++n;  // decrypt: advances whatever the tag says (noise.cpp:421)
  return true;
}

std::size_t Pipeline::submit_serial(const Message *messages, std::size_t n) {
  const bool dec = dir_ == Direction::Decrypt;
  Slot &sl = *slots_[fill_];
  // 1. bookkeeping in order (cheap): nonces, offsets, descriptors
  std::size_t k = 0, in_used = sl.in_used, out_used = sl.out_used;
  for (; k < n; ++k) {
    const Message &m = messages[k];
    // a refused message stops the batch before it; it throws when it comes first
    // (as its submit() would), so the messages ahead of it are never lost
    const bool bad_nonce = m.session >= nonces_.size() ||
                           nonces_[m.session] == std::numeric_limits<std::uint64_t>::max() - 1;
    const bool bad_len = dec ? (m.len < 16 || m.len > kMaxMessage) : m.len + 16 > kMaxMessage;
    if (bad_nonce || bad_len) {
      if (k > 0) break;
      const std::uint64_t nn = nonces_.at(m.session);
      if (nn == std::numeric_limits<std::uint64_t>::max() - 1)  // noise.cpp:398-400
        throw std::out_of_range("Nonce limit has been exceeded!");
      if (!dec) throw std::length_error("Noise message exceeds 65535 bytes");
      throw std::invalid_argument("Invalid MAC");
    }
    const std::uint64_t nn = nonces_[m.session];
    const std::size_t in_len = align16(m.len), out_len = dec ? align16(m.len - 16) : align16(m.len + 16);
    if (sl.nrec + k == opt_.slot_records || in_used + in_len > opt_.slot_bytes) break;
    sl.recs()[sl.nrec + k] = noise_gpu_record{in_used, out_used, nn, 0,
                                             (std::uint32_t)(dec ? m.len - 16 : m.len), 0,
                                             (std::uint32_t)m.session, 0};
    ++nonces_[m.session];  // decrypt: advances whatever the tag says (noise.cpp:421)
    in_used += in_len;
    out_used += out_len;
  }
  // 2. the byte copies, in parallel
  const std::size_t base = sl.nrec;
  pool_->run(k, [&](std::size_t lo, std::size_t hi) {
    for (std::size_t i = lo; i < hi; ++i)
      if (messages[i].len)
        stream_copy(sl.h + o_in_ + sl.recs()[base + i].in_off, messages[i].data, messages[i].len);
    stream_fence();  // visible to the H2D copy flush() issues
  });
  sl.nrec += k;
  sl.in_used = in_used;
  sl.out_used = out_used;
  return k;
}

// The bookkeeping of submit_batch in parallel as well as the copies (the
// serial loop above cost ~10 ns per message: at 256-byte messages it bound
// the Pipeline below the CPU).  Over the copy pool's T contiguous chunks of
// the messages that fit:
//   1. each thread finds its chunk's first refused message and its byte
//      total, and counts its messages per session;
//   2. the caller cuts the batch at the slot's record / byte capacity and the
//      first refused message, and gives every chunk its byte offsets and, per
//      session, its first nonce (the session's nonce + the earlier chunks'
//      counts) -- what consecutive submit() calls would have assigned;
//   3. each thread writes its descriptors and copies its messages.
// Falls back to the serial walk for few messages, a single thread, very many
// sessions (the counters are T x sessions) or a batch reaching a session's
// nonce limit (the exact exception order is the serial walk's).
std::size_t Pipeline::submit_batch(const Message *messages, std::size_t n) {
  const bool dec = dir_ == Direction::Decrypt;
  Slot &sl = *slots_[fill_];
  const std::size_t T = (std::size_t)pool_->nthr, S = nonces_.size();
  const std::size_t n0 = std::min(n, opt_.slot_records - sl.nrec);
  if (T == 1 || n0 < 4096 || S * T > (std::size_t(1) << 22)) return submit_serial(messages, n);
  auto in_len_of = [](std::size_t len) { return align16(len); };
  auto out_len_of = [dec](std::size_t len) { return dec ? align16(len - 16) : align16(len + 16); };
  auto refused = [&](const Message &m) {
    return m.session >= S || (dec ? (m.len < 16 || m.len > kMaxMessage) : m.len + 16 > kMaxMessage);
  };
  // the pool's chunk c of [0, len) is [len c / T, len (c + 1) / T), or all
  // of it in chunk 0 below 64 messages (CopyPool::run_idx passes c)
  // 1. per chunk: the first refused message, the input bytes before it
  //    (n0 >= 4096 here: every chunk is the T-way split the walk below uses)
  std::vector<std::size_t> bad(T, n0), bytes(T, 0);
  pool_->run_idx(n0, [&](std::size_t c, std::size_t lo, std::size_t hi) {
    std::size_t b = 0;
    for (std::size_t i = lo; i < hi; ++i) {
      if (refused(messages[i])) {
        bad[c] = i;
        break;
      }
      b += in_len_of(messages[i].len);
    }
    bytes[c] = b;
  });
  std::size_t k = n0;
  for (std::size_t c = 0; c < T; ++c) k = std::min(k, bad[c]);
  if (k == 0) return submit_serial(messages, n);  // throws exactly as submit() would
  {  // the byte capacity: walk the chunk where the running total passes it
    std::size_t used = sl.in_used;
    for (std::size_t c = 0; c < T; ++c) {
      const std::size_t lo = n0 * c / T, end = n0 * (c + 1) / T, hi = std::min(k, end);
      if (lo >= hi) break;
      if (hi == end && used + bytes[c] <= opt_.slot_bytes) {
        used += bytes[c];
        continue;
      }
      std::size_t i = lo;
      for (; i < hi; ++i) {
        const std::size_t l = in_len_of(messages[i].len);
        if (used + l > opt_.slot_bytes) break;
        used += l;
      }
      k = i;
      break;
    }
  }
  if (k == 0) return 0;  // the slot is full: flush() and call again
  // 2. per chunk of [0, k): its messages per session and its bytes
  sess_cnt_.assign(T * S, 0u);
  std::vector<std::size_t> in_b(T + 1, 0), out_b(T + 1, 0);
  pool_->run_idx(k, [&](std::size_t c, std::size_t lo, std::size_t hi) {
    std::uint32_t *cnt = sess_cnt_.data() + c * S;
    std::size_t bi = 0, bo = 0;
    for (std::size_t i = lo; i < hi; ++i) {
      ++cnt[messages[i].session];
      bi += in_len_of(messages[i].len);
      bo += out_len_of(messages[i].len);
    }
    in_b[c + 1] = bi;
    out_b[c + 1] = bo;
  });
  in_b[0] = sl.in_used;
  out_b[0] = sl.out_used;
  for (std::size_t c = 0; c < T; ++c) {
    in_b[c + 1] += in_b[c];
    out_b[c + 1] += out_b[c];
  }
  // each chunk's first nonce per session (the session's nonce + the earlier
  // chunks' counts); a batch that would reach a nonce limit takes the serial
  // walk, which throws at exactly the message submit() would
  constexpr std::uint64_t kLimit = std::numeric_limits<std::uint64_t>::max() - 1;
  std::vector<std::uint64_t> first(T * S), after(S);
  for (std::size_t s = 0; s < S; ++s) {
    std::uint64_t run = nonces_[s];
    for (std::size_t c = 0; c < T; ++c) {
      const std::uint32_t m = sess_cnt_[c * S + s];
      if (kLimit - run < m) return submit_serial(messages, n);
      first[c * S + s] = run;
      run += m;
    }
    after[s] = run;
  }
  // 3. descriptors and copies
  const std::size_t base = sl.nrec;
  pool_->run_idx(k, [&](std::size_t c, std::size_t lo, std::size_t hi) {
    std::uint64_t *nx = first.data() + c * S;
    std::size_t io = in_b[c], oo = out_b[c];
    noise_gpu_record *recs = sl.recs();
    for (std::size_t i = lo; i < hi; ++i) {
      const Message &m = messages[i];
      recs[base + i] = noise_gpu_record{io, oo, nx[m.session]++, 0,
                                        (std::uint32_t)(dec ? m.len - 16 : m.len), 0,
                                        (std::uint32_t)m.session, 0};
      if (m.len) stream_copy(sl.h + o_in_ + io, m.data, m.len);
      io += in_len_of(m.len);
      oo += out_len_of(m.len);
    }
    stream_fence();  // visible to the H2D copy flush() issues
  });
  nonces_.swap(after);  // decrypt: advances whatever the tags say (noise.cpp:421)
  sl.nrec += k;
  sl.in_used = in_b[T];
  sl.out_used = out_b[T];
  return k;
}

void Pipeline::copy_out(const Batch &b, std::uint8_t *const *dst) {
  pool_->run(b.size(), [&](std::size_t lo, std::size_t hi) {
    for (std::size_t i = lo; i < hi; ++i) stream_copy(dst[i], b.data(i), b.length(i));
    stream_fence();
  });
}

std::uint64_t Pipeline::flush() {
  Slot &sl = *slots_[fill_];
  if (sl.nrec == 0) return 0;
  const LaunchJob j{&sl, key_dirty_, nonces_.size()};
  key_dirty_ = j.nkeys;
  if (launcher_) {
    {
      std::lock_guard<std::mutex> lk(launcher_->mu);
      if (launcher_->err) std::rethrow_exception(launcher_->err);
      sl.enqueued = false;
      launcher_->q.push_back(j);
    }
    launcher_->cv.notify_one();
  } else {
    enqueue(j);
  }
  sl.in_flight = true;
  sl.ticket = ++tickets_;
  // move on; a slot still in flight is waited for here (back-pressure), and
  // its results are gone once refilled
  fill_ = (fill_ + 1) % slots_.size();
  Slot &nx = *slots_[fill_];
  if (nx.in_flight) {
    wait_enqueued(nx);
    hip_check(hipEventSynchronize(nx.done), "slot wait");
    nx.in_flight = false;
  }
  nx.nrec = nx.in_used = nx.out_used = 0;
  nx.ticket = 0;
  return sl.ticket;
}

void Pipeline::enqueue(const LaunchJob &j) {
  // flush() without the launcher thread runs this on the caller's thread:
  // the records call's scratch and companion stream are per (device, stream)
  const noise_amd::DeviceGuard on_dev(dev_);
  Slot &sl = *j.sl;
  const bool dec = dir_ == Direction::Decrypt;
  // Key rows reach the device table on the stream of the slot that first
  // needs them.  Every slot stream waits on keys_evt_ before its kernels, and
  // each upload waits on the previous one before recording keys_evt_ again,
  // so the event's latest record covers every row uploaded so far, whichever
  // slot stream carried it.
  if (keys_uploaded_) hip_check(hipStreamWaitEvent(sl.st, static_cast<hipEvent_t>(keys_evt_), 0), "key wait");
  if (j.key_lo < j.nkeys) {  // new sessions' keys (rows never change once written)
    hip_check(hipMemcpyAsync(d_keys_ + 32 * j.key_lo, h_keys_ + 32 * j.key_lo, 32 * (j.nkeys - j.key_lo),
                             hipMemcpyHostToDevice, sl.st), "key upload");
    hip_check(hipEventRecord(static_cast<hipEvent_t>(keys_evt_), sl.st), "key event");
    keys_uploaded_ = true;
  }
  hip_check(hipMemcpyAsync(sl.d, sl.h, sl.nrec * sizeof(noise_gpu_record), hipMemcpyHostToDevice, sl.st),
            "records H2D");
  if (sl.in_used)
    hip_check(hipMemcpyAsync(sl.d + o_in_, sl.h + o_in_, sl.in_used, hipMemcpyHostToDevice, sl.st),
              "messages H2D");
  const auto *d_recs = reinterpret_cast<const noise_gpu_record *>(sl.d);
  // the slot's plaintext bytes (the padded out / in images bound them):
  // lets a slot of few long messages take the load-balanced path
  const std::uint64_t len_sum = dec ? sl.out_used : sl.in_used;
  const int rc = dec ? noise_gpu_decrypt_records_sized(d_keys_, (std::uint32_t)j.nkeys, d_recs, sl.nrec,
                                                       sl.d + o_in_, sl.d + o_out_, nullptr, sl.d + o_st_,
                                                       len_sum, sl.st)
                     : noise_gpu_encrypt_records_sized(d_keys_, (std::uint32_t)j.nkeys, d_recs, sl.nrec,
                                                       sl.d + o_in_, sl.d + o_out_, nullptr, len_sum, sl.st);
  if (rc != NOISE_GPU_OK)
    throw std::runtime_error(std::string("noise-mi355x: ") + noise_gpu_strerror(rc) + ": " +
                             noise_gpu_last_error());
  if (sl.out_used)
    hip_check(hipMemcpyAsync(sl.h + o_out_, sl.d + o_out_, sl.out_used, hipMemcpyDeviceToHost, sl.st),
              "messages D2H");
  if (dec)
    hip_check(hipMemcpyAsync(sl.h + o_st_, sl.d + o_st_, sl.nrec, hipMemcpyDeviceToHost, sl.st),
              "status D2H");
  hip_check(hipEventRecord(sl.done, sl.st), "slot event");
}

Pipeline::Batch Pipeline::wait(std::uint64_t ticket) {
  Slot *sl = nullptr;
  for (Slot *c : slots_)
    if (c->ticket == ticket && ticket != 0) sl = c;
  if (!sl) throw std::logic_error("pipeline: ticket unknown or its slot was reused");
  if (sl->in_flight) {
    wait_enqueued(*sl);
    hip_check(hipEventSynchronize(sl->done), "slot wait");
    sl->in_flight = false;
  }
  Batch b;
  b.h_ = sl->h;
  b.n_ = sl->nrec;
  b.o_out_ = o_out_;
  b.o_st_ = o_st_;
  b.dec_ = dir_ == Direction::Decrypt;
  return b;
}

std::size_t Pipeline::Batch::session(std::size_t i) const {
  return reinterpret_cast<const noise_gpu_record *>(h_)[i].key_idx;
}
std::uint64_t Pipeline::Batch::nonce(std::size_t i) const {
  return reinterpret_cast<const noise_gpu_record *>(h_)[i].nonce;
}
bool Pipeline::Batch::ok(std::size_t i) const { return !dec_ || h_[o_st_ + i] == NOISE_GPU_REC_OK; }
const std::uint8_t *Pipeline::Batch::data(std::size_t i) const {
  return h_ + o_out_ + reinterpret_cast<const noise_gpu_record *>(h_)[i].out_off;
}
std::size_t Pipeline::Batch::length(std::size_t i) const {
  const std::size_t len = reinterpret_cast<const noise_gpu_record *>(h_)[i].len;
  return dec_ ? len : len + 16;
}

}  // namespace noise::transport
