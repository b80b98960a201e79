// transport_test.cpp -- noise::transport (framing + multi-session batcher)
// against the CPU oracle (oracle/liboracle.so: test infrastructure).
//
//   transport_test <sessions> <messages> <seed>
//   transport_test pipeline <sessions> <messages> <seed>  the same through
//       noise::transport::Pipeline (small slots: many flushes in flight,
//       full-slot retries, ticket reuse), ciphertexts vs the oracle and vs
//       the Batcher's, decrypt round trip with tampered records
//   transport_test keyrace <sessions>   Pipeline key-table ordering: slot A
//       uploads a large table of new sessions' keys, slot B (another stream,
//       no upload of its own) is flushed right after with messages of the
//       last sessions; B's ciphertexts must match the oracle
//   transport_test resident_race <sessions> [seconds]   Pipeline work on one
//       thread while another sends resident single-record traffic: the
//       Pipeline must not wait for the resident instance
//   transport_test bench <batcher|pipeline> <sessions> <messages> <len> [threads]
//       host-resident throughput, encrypt then decrypt, GiB/s of plaintext;
//       threads > 1: Pipeline::submit_batch / copy_out over that many copy threads
// Sessions get random keys and start nonces; messages (0..2000 bytes, some
// 65519) are submitted interleaved, encrypted in ONE batch, checked bit-exact
// against oracle_noise_encrypt with each session's nonce sequence, framed per
// session into a byte stream, re-read through a Deframer fed in random-size
// chunks, decrypted in ONE batch (one record tampered per 97) and compared.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <deque>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "noise_amd/transport.hpp"
#include "noise_gpu.h"

extern "C" {
void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad, size_t ad_len,
                          const uint8_t *pt, size_t len, uint8_t *out);
}

using bytes = std::vector<std::uint8_t>;
namespace nt = noise::transport;

static int run_pipeline(int S, int M, std::uint64_t seed) {
  std::mt19937_64 rng(seed);
  int fails = 0;
  auto check = [&](bool c, const char *what, long i) {
    if (!c && fails++ < 20) std::printf("FAIL %s (%ld)\n", what, i);
  };
  nt::Pipeline::Options o;
  o.launch_thread = seed % 2 == 0;  // odd seeds: flush() issues the HIP work itself
  o.slot_bytes = 256 << 10;  // small slots: many flushes, full-slot retries
  o.slot_records = 97;
  o.depth = 3;
  nt::Pipeline enc(nt::Pipeline::Direction::Encrypt, o), dec(nt::Pipeline::Direction::Decrypt, o);
  nt::Batcher ref(nt::Batcher::Direction::Encrypt);
  std::vector<std::array<std::uint8_t, 32>> keys(S);
  std::vector<std::uint64_t> n0(S);
  for (int s = 0; s < S; ++s) {
    for (auto &b : keys[s]) b = (std::uint8_t)rng();
    n0[s] = rng() % 3 == 0 ? (1ull << 32) - 2 + (rng() % 5) : rng() % 1000;
    noise::CipherState cs;
    cs.initialize_key(keys[s]);
    cs.set_nonce(n0[s]);
    check(enc.add_session(cs) == (std::size_t)s && dec.add_session(cs) == (std::size_t)s &&
              ref.add_session(cs) == (std::size_t)s, "session id", s);
  }
  std::vector<int> sess(M);
  std::vector<bytes> pt(M), ct(M);
  for (int i = 0; i < M; ++i) {
    sess[i] = (int)(rng() % S);
    const std::size_t len = rng() % 41 == 0 ? 65519 : rng() % 3 == 0 ? 1024 : rng() % 2001;
    pt[i].resize(len);
    for (auto &b : pt[i]) b = (std::uint8_t)rng();
    ref.submit(sess[i], pt[i]);
  }
  // encrypt through the ring: a flush refills the slot of the ticket two
  // flushes back, so at most depth - 2 tickets may stay unconsumed across it
  std::deque<std::pair<std::uint64_t, int>> outstanding;  // ticket, first message index
  int next_i = 0, done = 0, flushes = 0;
  auto drain = [&](std::size_t keep) {
    while (outstanding.size() > keep) {
      auto [t, first] = outstanding.front();
      outstanding.pop_front();
      const nt::Pipeline::Batch b = enc.wait(t);
      for (std::size_t j = 0; j < b.size(); ++j) {
        const int i = first + (int)j;
        check(b.session(j) == (std::size_t)sess[i] && b.ok(j) && b.length(j) == pt[i].size() + 16,
              "pipeline result header", i);
        ct[i].assign(b.data(j), b.data(j) + b.length(j));
        ++done;
      }
    }
  };
  int first = 0;
  while (next_i < M) {
    if (enc.submit(sess[next_i], pt[next_i].data(), pt[next_i].size())) {
      ++next_i;
      continue;
    }
    outstanding.push_back({enc.flush(), first});
    ++flushes;
    first = next_i;
    drain(o.depth - 2);  // the next flush reuses the slot of ticket t-2
  }
  if (enc.pending()) {
    outstanding.push_back({enc.flush(), first});
    ++flushes;
  }
  drain(0);
  check(done == M, "all results", done);
  bool threw = false;
  try {
    (void)enc.wait(1);  // long since reused
  } catch (const std::logic_error &) {
    threw = true;
  }
  check(threw || flushes <= o.depth, "stale ticket refused", flushes);
  const std::vector<nt::Batcher::Result> want = ref.flush();
  std::vector<std::uint64_t> next(n0);
  bytes w(65535 + 16);
  for (int i = 0; i < M; ++i) {
    oracle_noise_encrypt(keys[sess[i]].data(), next[sess[i]]++, nullptr, 0, pt[i].data(), pt[i].size(),
                         w.data());
    check(ct[i].size() == pt[i].size() + 16 && std::memcmp(ct[i].data(), w.data(), ct[i].size()) == 0,
          "pipeline ciphertext vs oracle", i);
    check(ct[i] == want[i].msg, "pipeline vs batcher", i);
  }
  for (int s = 0; s < S; ++s) check(enc.nonce(s) == next[s], "encrypt nonce advance", s);
  // decrypt, tampering every 89th; one flush at a time
  std::vector<bytes> back(M);
  std::vector<bool> okv(M);
  int i0 = 0;
  for (int i = 0; i <= M; ++i) {
    bytes m;
    if (i < M) {
      m = ct[i];
      if (i % 89 == 3) m[rng() % m.size()] ^= 0x10;
      if (dec.submit(sess[i], m.data(), m.size())) continue;
    }
    const std::uint64_t t = dec.flush();
    if (t) {
      const nt::Pipeline::Batch b = dec.wait(t);
      for (std::size_t j = 0; j < b.size(); ++j) {
        okv[i0 + j] = b.ok(j);
        if (b.ok(j)) back[i0 + j].assign(b.data(j), b.data(j) + b.length(j));
      }
      i0 += (int)b.size();
    }
    if (i < M) check(dec.submit(sess[i], m.data(), m.size()), "submit after flush", i);
  }
  check(i0 == M, "decrypt count", i0);
  for (int i = 0; i < M; ++i) {
    if (i % 89 == 3) check(!okv[i], "tampered rejected", i);
    else check(okv[i] && back[i] == pt[i], "decrypt round trip", i);
  }
  for (int s = 0; s < S; ++s) check(dec.nonce(s) == next[s], "decrypt nonce advance", s);
  std::printf("pipeline sessions %d messages %d flushes %d: %s (%d failures)\n", S, M, flushes,
              fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}

// Pipeline::submit_batch / copy_out (4 copy threads): ragged chunks of
// messages (1..300, crossing slot boundaries), ciphertexts vs the oracle,
// then decrypt back through batches with tampered records.
// slot_records >= 4096 with several copy threads takes submit_batch's
// parallel bookkeeping (chunked session counts / nonce scan); the default
// tiny slots its serial walk
static int run_pipeline_batch(int S, int M, std::uint64_t seed, std::size_t slot_records = 97,
                              std::size_t slot_bytes = 256 << 10, std::size_t maxlen = 3000,
                              int maxbatch = 300, int threads = 4, int big_every = 29) {
  std::mt19937_64 rng(seed);
  int fails = 0;
  auto check = [&](bool c, const char *what, long i) {
    if (!c && fails++ < 20) std::printf("FAIL %s (%ld)\n", what, i);
  };
  nt::Pipeline::Options o;
  o.launch_thread = seed % 2 == 0;  // odd seeds: flush() issues the HIP work itself
  o.slot_bytes = slot_bytes;
  o.slot_records = slot_records;
  o.depth = 3;
  o.copy_threads = threads;  // > 64 with a byte cut below it: chunks that share a first index
  nt::Pipeline enc(nt::Pipeline::Direction::Encrypt, o), dec(nt::Pipeline::Direction::Decrypt, o);
  std::vector<std::array<std::uint8_t, 32>> keys(S);
  std::vector<std::uint64_t> n0(S);
  for (int s = 0; s < S; ++s) {
    for (auto &b : keys[s]) b = (std::uint8_t)rng();
    n0[s] = rng() % 1000;
    noise::CipherState cs;
    cs.initialize_key(keys[s]);
    cs.set_nonce(n0[s]);
    enc.add_session(cs);
    dec.add_session(cs);
  }
  std::vector<bytes> pt(M), ct(M), back(M);
  std::vector<nt::Pipeline::Message> msgs(M);
  for (int i = 0; i < M; ++i) {
    // every ~big_every-th message is a maximum-size one (0: none)
    pt[i].resize(big_every > 0 && rng() % (unsigned)big_every == 0 ? 65519 : rng() % maxlen);
    for (auto &b : pt[i]) b = (std::uint8_t)rng();
    msgs[i] = {(std::size_t)(rng() % S), pt[i].data(), pt[i].size()};
  }
  // one direction through the ring: batches of random size, results copied out
  auto run = [&](nt::Pipeline &p, std::vector<bytes> &out, bool decrypt, std::vector<bool> *okv) {
    std::deque<std::pair<std::uint64_t, int>> q;
    std::vector<std::uint8_t *> dst(o.slot_records);
    auto take = [&](std::size_t keep) {
      while (q.size() > keep) {
        auto [t, f] = q.front();
        q.pop_front();
        const nt::Pipeline::Batch b = p.wait(t);
        for (std::size_t j = 0; j < b.size(); ++j) {
          out[f + j].assign(b.length(j), 0);
          dst[j] = out[f + j].data();
          if (okv) (*okv)[f + j] = b.ok(j);
        }
        p.copy_out(b, dst.data());
      }
    };
    int i = 0, first = 0;
    while (i < M) {
      const int want = std::min<int>(M - i, 1 + (int)(rng() % maxbatch));
      const std::size_t k = p.submit_batch(msgs.data() + i, (std::size_t)want);
      i += (int)k;
      if (k < (std::size_t)want) {
        q.push_back({p.flush(), first});
        first = i;
        take(o.depth - 2);
      }
    }
    if (p.pending()) q.push_back({p.flush(), first});
    take(0);
    (void)decrypt;
  };
  run(enc, ct, false, nullptr);
  std::vector<std::uint64_t> next(n0);
  bytes w(65535 + 16);
  for (int i = 0; i < M; ++i) {
    const std::size_t s = msgs[i].session;
    oracle_noise_encrypt(keys[s].data(), next[s]++, nullptr, 0, pt[i].data(), pt[i].size(), w.data());
    check(ct[i].size() == pt[i].size() + 16 && std::memcmp(ct[i].data(), w.data(), ct[i].size()) == 0,
          "batched ciphertext vs oracle", i);
  }
  for (int s = 0; s < S; ++s) check(enc.nonce(s) == next[s], "batched nonce advance", s);
  for (int i = 0; i < M; ++i) {
    if (i % 71 == 9) ct[i][rng() % ct[i].size()] ^= 0x02;
    msgs[i].data = ct[i].data();
    msgs[i].len = ct[i].size();
  }
  std::vector<bool> okv(M);
  run(dec, back, true, &okv);
  for (int i = 0; i < M; ++i) {
    if (i % 71 == 9) check(!okv[i], "batched tampered rejected", i);
    else check(okv[i] && back[i] == pt[i], "batched decrypt round trip", i);
  }
  std::printf("pipeline_batch sessions %d messages %d: %s (%d failures)\n", S, M, fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}

static int run_keyrace(int S) {
  int fails = 0;
  std::mt19937_64 rng(99);
  nt::Pipeline::Options o;
  o.depth = 2;
  o.slot_bytes = 4 << 20;
  o.slot_records = 4096;
  nt::Pipeline enc(nt::Pipeline::Direction::Encrypt, o);
  std::vector<std::array<std::uint8_t, 32>> keys(S);
  for (int s = 0; s < S; ++s) {
    for (auto &b : keys[s]) b = (std::uint8_t)rng();
    noise::CipherState cs;
    cs.initialize_key(keys[s]);
    enc.add_session(cs);
  }
  bytes pt(1024);
  for (auto &b : pt) b = (std::uint8_t)rng();
  // slot A: one message of session 0 -> uploads all S key rows on A's stream
  enc.submit(0, pt.data(), pt.size());
  const std::uint64_t ta = enc.flush();
  // slot B, flushed at once: messages of the sessions uploaded last
  const int M = 2048;
  for (int i = 0; i < M; ++i)
    if (!enc.submit(S - 1 - i, pt.data(), pt.size()) && fails++ < 10) std::printf("FAIL submit %d\n", i);
  const std::uint64_t tb = enc.flush();
  const nt::Pipeline::Batch b = enc.wait(tb);
  if (b.size() != (std::size_t)M && fails++ < 10) std::printf("FAIL batch size %zu\n", b.size());
  bytes want(1024 + 16);
  for (int i = 0; i < M; ++i) {
    const int s = S - 1 - i;
    oracle_noise_encrypt(keys[s].data(), 0, nullptr, 0, pt.data(), pt.size(), want.data());
    if (b.length(i) != want.size() || std::memcmp(b.data(i), want.data(), want.size()) != 0)
      if (fails++ < 10) std::printf("FAIL keyrace record %d (session %d)\n", i, s);
  }
  (void)ta;
  std::printf("keyrace sessions %d messages %d: %s (%d failures)\n", S, M, fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}

// Resident traffic beside batch work: thread A turns on the
// resident latency mode and sends 1 KiB records back to back (gaps of a few
// microseconds, far below the instance's idle exit), thread B meanwhile builds
// a Pipeline, adds S sessions (the key table doubles from 1024 rows up) and
// encrypts growing batches through it (the records scratch of a slot stream
// grows), checked against the oracle.  Nothing B does may wait for every
// stream of the device (hipDeviceSynchronize / hipFree would wait for A's
// instance, i.e. until A stops): B must finish while A is still sending.
// Prints B's time and A's record count; fails if B outlived A's traffic.
static int run_resident_race(int S, double a_max_s) {
  using clk = std::chrono::steady_clock;
  int fails = 0;
  std::atomic<bool> b_done{false};
  std::atomic<long> a_records{0};
  std::atomic<int> a_err{0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::thread ta([&] {
    (void)hipSetDevice(dev);
    if (noise_gpu_set_resident(1, 0) != NOISE_GPU_OK) {
      a_err = 1;
      return;
    }
    std::array<std::uint8_t, 32> key{};
    for (int i = 0; i < 32; ++i) key[i] = (std::uint8_t)(i + 1);
    bytes buf(1024 + 16), pt(1024), want(1024 + 16);
    for (std::size_t i = 0; i < pt.size(); ++i) pt[i] = (std::uint8_t)(i * 7);
    const auto t0 = clk::now();
    std::uint64_t n = 0;
    while (!b_done.load() && std::chrono::duration<double>(clk::now() - t0).count() < a_max_s) {
      std::memcpy(buf.data(), pt.data(), pt.size());
      if (noise_gpu_encrypt_host(key.data(), n, nullptr, 0, buf.data(), pt.size()) != NOISE_GPU_OK) {
        a_err = 2;
        break;
      }
      if ((n & 1023u) == 0) {  // now and then against the oracle
        oracle_noise_encrypt(key.data(), n, nullptr, 0, pt.data(), pt.size(), want.data());
        if (buf != want) a_err = 3;
      }
      ++n;
      ++a_records;
    }
    (void)noise_gpu_set_resident(0, 0);
  });
  while (a_records.load() < 200 && !a_err.load()) std::this_thread::yield();
  const auto t0 = clk::now();
  double tb = 0;
  std::vector<double> phase;  // seconds since t0: Pipeline built, sessions added, each flush done
  {
    std::mt19937_64 rng(7);
    nt::Pipeline::Options o;
    o.slot_bytes = 64 << 20;
    o.slot_records = 65536;
    nt::Pipeline enc(nt::Pipeline::Direction::Encrypt, o);
    phase.push_back(std::chrono::duration<double>(clk::now() - t0).count());
    std::vector<std::array<std::uint8_t, 32>> keys(S);
    for (int s = 0; s < S; ++s) {
      for (auto &b : keys[s]) b = (std::uint8_t)rng();
      noise::CipherState cs;
      cs.initialize_key(keys[s]);
      enc.add_session(cs);
    }
    phase.push_back(std::chrono::duration<double>(clk::now() - t0).count());
    std::vector<std::uint64_t> next(S, 0);
    bytes pt(4096), want(4096 + 16);
    for (auto &b : pt) b = (std::uint8_t)rng();
    // five flushes; the fifth, the largest, lands on the first slot's stream
    // again and grows its records scratch
    for (int f = 0; f < 5; ++f) {
      const int M = f < 4 ? 2500 : 30000;
      std::vector<int> sess(M);
      std::vector<std::size_t> len(M);
      std::vector<std::uint64_t> nonce(M);
      for (int i = 0; i < M; ++i) {
        sess[i] = (int)(rng() % S);
        len[i] = i % 7 == 0 ? 4096 : 1024;
        nonce[i] = next[sess[i]]++;
        if (!enc.submit(sess[i], pt.data(), len[i]) && fails++ < 10) std::printf("FAIL submit %d\n", i);
      }
      const nt::Pipeline::Batch b = enc.wait(enc.flush());
      for (int i = 0; i < M; i += 13) {
        oracle_noise_encrypt(keys[sess[i]].data(), nonce[i], nullptr, 0, pt.data(), len[i], want.data());
        if (b.length(i) != len[i] + 16 || std::memcmp(b.data(i), want.data(), len[i] + 16) != 0)
          if (fails++ < 10) std::printf("FAIL record %d of flush %d\n", i, f);
      }
      phase.push_back(std::chrono::duration<double>(clk::now() - t0).count());
    }
    tb = std::chrono::duration<double>(clk::now() - t0).count();
    b_done = true;  // A stops; the Pipeline's destructor (hipHostFree) may wait for that
  }
  ta.join();
  if (a_err.load() && fails++ < 10) std::printf("FAIL resident thread error %d\n", a_err.load());
  if (tb >= a_max_s * 0.9 && fails++ < 10)
    std::printf("FAIL the Pipeline work took %.2f s: it waited for the resident traffic\n", tb);
  std::printf("{\"resident_race\": \"%s\", \"sessions\": %d, \"pipeline_s\": %.3f, "
              "\"resident_records_meanwhile\": %ld, \"failures\": %d, \"phases_s\": [",
              fails ? "FAIL" : "ok", S, tb, a_records.load(), fails);
  for (std::size_t i = 0; i < phase.size(); ++i) std::printf("%s%.3f", i ? ", " : "", phase[i]);
  std::printf("]}\n");
  return fails ? 1 : 0;
}

// Which HIP runtime calls wait for a resident instance on another thread's
// stream?  For each call: start steady resident traffic on a second thread,
// time the call, stop the traffic (after at most `cap_s`).  A call that
// waits for every stream of the device takes ~cap_s.
static int run_resident_probe(double cap_s) {
  using clk = std::chrono::steady_clock;
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipStream_t st = nullptr;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  struct Op {
    const char *name;
    std::function<void()> fn;
  };
  void *hp = nullptr, *dp = nullptr, *ap = nullptr;
  std::vector<Op> ops = {
      {"hipHostMalloc", [&] { (void)hipHostMalloc(&hp, 64 << 20, hipHostMallocDefault); }},
      {"hipMalloc", [&] { (void)hipMalloc(&dp, 64 << 20); }},
      {"hipMallocAsync", [&] { (void)hipMallocAsync(&ap, 64 << 20, st); (void)hipStreamSynchronize(st); }},
      {"hipMemcpyAsync+streamsync", [&] {
         (void)hipMemcpyAsync(dp, hp, 1 << 20, hipMemcpyHostToDevice, st);
         (void)hipStreamSynchronize(st);
       }},
      {"hipMemcpy", [&] { (void)hipMemcpy(dp, hp, 1 << 20, hipMemcpyHostToDevice); }},
      {"hipMemset", [&] { (void)hipMemset(dp, 0, 1 << 20); }},
      {"hipFreeAsync", [&] { (void)hipFreeAsync(ap, st); (void)hipStreamSynchronize(st); }},
      {"hipFree", [&] { (void)hipFree(dp); }},
      {"hipHostFree", [&] { (void)hipHostFree(hp); }},
      {"hipStreamCreate+Destroy", [&] {
         hipStream_t s2;
         (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
         (void)hipStreamDestroy(s2);
       }},
      {"hipStreamCreate+hipMallocAsync+sync", [&] {
         hipStream_t s2;
         void *q = nullptr;
         (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
         (void)hipMallocAsync(&q, 64 << 20, s2);
         (void)hipStreamSynchronize(s2);
         (void)hipFreeAsync(q, s2);
         (void)hipStreamSynchronize(s2);
         (void)hipStreamDestroy(s2);
       }},
      {"hipStreamCreate x6 + kernel-free sync", [&] {
         hipStream_t s2[6];
         for (auto &x : s2) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
         for (auto &x : s2) (void)hipStreamSynchronize(x);
         for (auto &x : s2) (void)hipStreamDestroy(x);
       }},
      {"hipEventCreate+Destroy", [&] {
         hipEvent_t e;
         (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
         (void)hipEventDestroy(e);
       }},
  };
  int pools = -1;
  const hipError_t pe = hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, dev);
  std::printf("{\"resident_probe_cap_s\": %.1f, \"memory_pools_attr\": %d, \"attr_rc\": %d", cap_s, pools,
              (int)pe);
  for (const Op &op : ops) {
    std::atomic<bool> stop{false};
    std::atomic<long> recs{0};
    std::thread ta([&] {
      (void)hipSetDevice(dev);
      (void)noise_gpu_set_resident(1, 0);
      std::array<std::uint8_t, 32> key{};
      key[0] = 1;
      bytes buf(64 + 16);
      const auto t0 = clk::now();
      for (std::uint64_t n = 0; !stop.load() && std::chrono::duration<double>(clk::now() - t0).count() < cap_s; ++n) {
        (void)noise_gpu_encrypt_host(key.data(), n, nullptr, 0, buf.data(), 64);
        ++recs;
      }
      std::fprintf(stderr, "probe: traffic stops\n");
      const int rc = noise_gpu_set_resident(0, 0);
      std::fprintf(stderr, "probe: resident off rc %d (%s)\n", rc, noise_gpu_last_error());
      if (std::getenv("PROBE_THREAD_RELEASE")) {
        const int rc2 = noise_gpu_thread_release();
        std::fprintf(stderr, "probe: thread release rc %d\n", rc2);
      }
    });
    while (recs.load() < 200) std::this_thread::yield();
    std::fprintf(stderr, "probe: %s ...\n", op.name);
    const auto t0 = clk::now();
    op.fn();
    const double t = std::chrono::duration<double>(clk::now() - t0).count();
    std::fprintf(stderr, "probe: %s %.4f s (%ld resident records so far)\n", op.name, t, recs.load());
    stop = true;
    ta.join();
    std::fprintf(stderr, "probe: traffic thread joined\n");
    std::printf(", \"%s\": %.4f", op.name, t);
    std::fflush(stdout);
  }
  std::printf("}\n");
  (void)hipStreamDestroy(st);
  return 0;
}

// A live resident instance for `secs` seconds (tools/gpu/r4_resident_cost.sh
// runs the batch benches beside it).  busy: 0 = a record every 5 ms, 1 = back
// to back, 2 = one record, then the instance just polls; 3 = no instance, an
// idle HIP context only (what a second process on the GPU costs by itself)
static int run_resident_hold(double secs, int busy) {
  using clk = std::chrono::steady_clock;
  if (busy == 3 && hipFree(nullptr) != hipSuccess) return 1;
  if (busy != 3 && noise_gpu_set_resident(1, 10000000) != NOISE_GPU_OK) return 1;
  std::array<std::uint8_t, 32> key{};
  key[0] = 9;
  bytes buf(1024 + 16);
  long n = 0;
  const auto t0 = clk::now();
  const char *stop_file = std::getenv("RESIDENT_HOLD_STOP");  // leave early once it exists
  while (std::chrono::duration<double>(clk::now() - t0).count() < secs) {
    if (busy <= 1 || (busy == 2 && n == 0)) {
      if (noise_gpu_encrypt_host(key.data(), (std::uint64_t)n, nullptr, 0, buf.data(), 1024) != NOISE_GPU_OK)
        return 2;
      ++n;
    } else {
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    if (!busy) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (stop_file && (busy >= 2 || (n & 255) == 0)) {
      if (FILE *f = std::fopen(stop_file, "r")) {
        std::fclose(f);
        break;
      }
    }
  }
  const double t = std::chrono::duration<double>(clk::now() - t0).count();
  if (busy != 3) (void)noise_gpu_set_resident(0, 0);
  if (n == 0) n = 1;
  std::printf("{\"resident_hold\": %d, \"records\": %ld, \"seconds\": %.2f, \"us_per_record\": %.3f}\n",
              busy, n, t, t / (double)n * 1e6);
  return 0;
}

// Host-resident throughput: M messages of len bytes from one source buffer
// (the "socket reads"), encrypt then decrypt, results checksummed (touched).
static int run_bench(const std::string &mode, int S, long M, std::size_t len, int threads = 1,
                     int depth = 0, int launch = 1, std::size_t slot_records = 0) {
  std::mt19937_64 rng(7);
  bytes src((std::size_t)M * len);
  for (std::size_t i = 0; i < src.size(); i += 8) {
    const std::uint64_t v = rng();
    std::memcpy(src.data() + i, &v, std::min<std::size_t>(8, src.size() - i));
  }
  std::vector<noise::CipherState> cs(S);
  for (int s = 0; s < S; ++s) {
    std::array<std::uint8_t, 32> k;
    for (auto &b : k) b = (std::uint8_t)rng();
    cs[s].initialize_key(k);
  }
  using clk = std::chrono::steady_clock;
  std::uint64_t sum = 0;
  double secs[2] = {0, 0};
  double phase[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};  // submit_batch, flush, wait, copy_out
  bytes ctall((std::size_t)M * (len + 16)), ptall(threads > 1 ? (std::size_t)M * len : 0);
  // long-lived objects, as in a server: built (pinned slots, key upload)
  // outside the timed region
  nt::Pipeline::Options popt;
  popt.copy_threads = threads;
  if (depth > 0) popt.depth = depth;
  popt.launch_thread = launch != 0;
  if (slot_records) popt.slot_records = slot_records;
  // results consumed depth - 2 flushes after their own: the next flush
  // reuses the slot depth - 1 back, and depth - 2 slots stay in flight
  const std::size_t keep = (std::size_t)popt.depth - 2;
  nt::Pipeline penc(nt::Pipeline::Direction::Encrypt, popt), pdec(nt::Pipeline::Direction::Decrypt, popt);
  for (int s = 0; s < S; ++s) {
    penc.add_session(cs[s]);
    pdec.add_session(cs[s]);
  }
  for (int pass = 0; pass < 3; ++pass) {  // pass 0 warms up (kernels, scratch)
    for (int d = 0; d < 2; ++d) {
      const bool dec = d == 1;
      const std::size_t ilen = dec ? len + 16 : len;
      const std::uint8_t *in = dec ? ctall.data() : src.data();
      const auto t0 = clk::now();
      if (mode == "batcher") {
        nt::Batcher b(dec ? nt::Batcher::Direction::Decrypt : nt::Batcher::Direction::Encrypt);
        for (int s = 0; s < S; ++s) b.add_session(cs[s]);
        const long per = 1 << 16;
        for (long i0 = 0; i0 < M; i0 += per) {
          for (long i = i0; i < std::min(M, i0 + per); ++i)
            b.submit(i % S, bytes(in + i * ilen, in + (i + 1) * ilen));
          const auto r = b.flush();
          for (std::size_t j = 0; j < r.size(); ++j) {
            if (!dec) std::memcpy(ctall.data() + (i0 + j) * (len + 16), r[j].msg.data(), len + 16);
            sum += r[j].msg[0];
          }
        }
      } else if (threads > 1) {  // batched submit / copy-out over the pipeline's copy threads
        nt::Pipeline &p = dec ? pdec : penc;
        std::deque<std::pair<std::uint64_t, long>> q;
        std::vector<nt::Pipeline::Message> msgs(M);
        for (long i = 0; i < M; ++i) msgs[i] = {(std::size_t)(i % S), in + i * ilen, ilen};
        std::vector<std::uint8_t *> dst(popt.slot_records);
        auto take = [&](std::size_t keep) {
          while (q.size() > keep) {
            auto [t, f] = q.front();
            q.pop_front();
            const auto w0 = clk::now();
            const nt::Pipeline::Batch b = p.wait(t);
            const auto w1 = clk::now();
            phase[d][2] += std::chrono::duration<double>(w1 - w0).count();
            // results consumed: every message copied out (as a send() would), in parallel
            for (std::size_t j = 0; j < b.size(); ++j)
              dst[j] = dec ? ptall.data() + (f + j) * len : ctall.data() + (f + j) * (len + 16);
            p.copy_out(b, dst.data());
            if (dec)
              for (std::size_t j = 0; j < b.size(); ++j)
                if (!b.ok(j)) throw std::runtime_error("bench: decrypt failed");
            phase[d][3] += std::chrono::duration<double>(clk::now() - w1).count();
          }
        };
        long i = 0, first = 0;
        while (i < M) {
          const auto s0 = clk::now();
          const std::size_t k = p.submit_batch(msgs.data() + i, (std::size_t)(M - i));
          const auto s1 = clk::now();
          phase[d][0] += std::chrono::duration<double>(s1 - s0).count();
          i += (long)k;
          if (i < M) {
            q.push_back({p.flush(), first});
            phase[d][1] += std::chrono::duration<double>(clk::now() - s1).count();
            first = i;
            take(keep);
          }
        }
        q.push_back({p.flush(), first});
        take(0);
      } else {
        nt::Pipeline &p = dec ? pdec : penc;
        std::deque<std::pair<std::uint64_t, long>> q;
        long first = 0;
        auto take = [&](std::size_t keep) {
          while (q.size() > keep) {
            auto [t, f] = q.front();
            q.pop_front();
            const nt::Pipeline::Batch b = p.wait(t);
            for (std::size_t j = 0; j < b.size(); ++j) {
              if (!dec) std::memcpy(ctall.data() + (f + j) * (len + 16), b.data(j), len + 16);
              else if (!b.ok(j)) throw std::runtime_error("bench: decrypt failed");
              sum += b.data(j)[0];
            }
          }
        };
        for (long i = 0; i < M;) {
          if (p.submit(i % S, in + i * ilen, ilen)) {
            ++i;
            continue;
          }
          q.push_back({p.flush(), first});
          first = i;
          take(keep);
        }
        q.push_back({p.flush(), first});
        take(0);
      }
      const double t = std::chrono::duration<double>(clk::now() - t0).count();
      if (pass > 0) secs[d] += t;
    }
  }
  if (threads > 1) {  // the copied-out results, checked once outside the timed region
    if (ptall != src) throw std::runtime_error("bench: batched round trip differs");
    for (long i = 0; i < M; ++i) sum += ctall[(std::size_t)i * (len + 16)] + ptall[(std::size_t)i * len];
  }
  const double gib = (double)M * len * 2 / (1u << 30);  // two timed passes per direction
  std::printf("{\"mode\": \"%s\", \"copy_threads\": %d, \"depth\": %d, \"launch_thread\": %d, \"slot_records\": %zu, \"sessions\": %d, \"messages\": %ld, "
              "\"len\": %zu, \"encrypt_gib_s\": %.2f, \"decrypt_gib_s\": %.2f, "
              "\"phases_ms\": {\"encrypt\": [%.1f, %.1f, %.1f, %.1f], \"decrypt\": [%.1f, %.1f, %.1f, %.1f], "
              "\"order\": \"submit_batch, flush, wait, copy_out + status check (batched mode; all passes)\"}, "
              "\"checksum\": %llu}\n",
              mode.c_str(), threads, popt.depth, (int)popt.launch_thread, popt.slot_records, S, M, len, gib / secs[0], gib / secs[1], phase[0][0] * 1e3,
              phase[0][1] * 1e3, phase[0][2] * 1e3, phase[0][3] * 1e3, phase[1][0] * 1e3, phase[1][1] * 1e3,
              phase[1][2] * 1e3, phase[1][3] * 1e3, (unsigned long long)sum);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "pipeline")
    return run_pipeline(std::atoi(argv[2]), std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 0));
  if (argc > 1 && std::string(argv[1]) == "keyrace") return run_keyrace(std::atoi(argv[2]));
  if (argc > 1 && std::string(argv[1]) == "resident_hold")
    return run_resident_hold(std::atof(argv[2]), std::atoi(argv[3]));
  if (argc > 1 && std::string(argv[1]) == "resident_probe")
    return run_resident_probe(argc > 2 ? std::atof(argv[2]) : 3.0);
  if (argc > 1 && std::string(argv[1]) == "resident_race")
    return run_resident_race(std::atoi(argv[2]), argc > 3 ? std::atof(argv[3]) : 60.0);
  if (argc > 1 && std::string(argv[1]) == "pipeline_batch") {
    if (argc > 8)  // slot_records slot_bytes maxlen maxbatch [copy threads]
      return run_pipeline_batch(std::atoi(argv[2]), std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 0),
                                std::strtoull(argv[5], nullptr, 0), std::strtoull(argv[6], nullptr, 0),
                                std::strtoull(argv[7], nullptr, 0), std::atoi(argv[8]),
                                argc > 9 ? std::atoi(argv[9]) : 4, argc > 10 ? std::atoi(argv[10]) : 29);
    return run_pipeline_batch(std::atoi(argv[2]), std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 0));
  }
  if (argc > 1 && std::string(argv[1]) == "bench")
    return run_bench(argv[2], std::atoi(argv[3]), std::atol(argv[4]), std::strtoul(argv[5], nullptr, 0),
                     argc > 6 ? std::atoi(argv[6]) : 1, argc > 7 ? std::atoi(argv[7]) : 0,
                     argc > 8 ? std::atoi(argv[8]) : 1, argc > 9 ? std::strtoul(argv[9], nullptr, 0) : 0);
  const int S = argc > 1 ? std::atoi(argv[1]) : 100;
  const int M = argc > 2 ? std::atoi(argv[2]) : 1000;
  std::mt19937_64 rng(argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 1);
  int fails = 0;
  auto check = [&](bool c, const char *what, int i) {
    if (!c && fails++ < 20) std::printf("FAIL %s (%d)\n", what, i);
  };
  nt::Batcher enc(nt::Batcher::Direction::Encrypt), dec(nt::Batcher::Direction::Decrypt);
  std::vector<std::array<std::uint8_t, 32>> keys(S);
  std::vector<std::uint64_t> n0(S);
  for (int s = 0; s < S; ++s) {
    for (auto &b : keys[s]) b = (std::uint8_t)rng();
    n0[s] = rng() % 3 == 0 ? (1ull << 32) - 2 + (rng() % 5) : rng() % 1000;
    noise::CipherState cs;
    cs.initialize_key(keys[s]);
    cs.set_nonce(n0[s]);
    check(enc.add_session(cs) == (std::size_t)s, "session id", s);
    check(dec.add_session(cs) == (std::size_t)s, "session id", s);
  }
  std::vector<int> sess(M);
  std::vector<bytes> pt(M);
  for (int i = 0; i < M; ++i) {
    sess[i] = (int)(rng() % S);
    const std::size_t len = rng() % 23 == 0 ? 65519 : rng() % 2001;
    pt[i].resize(len);
    for (auto &b : pt[i]) b = (std::uint8_t)rng();
    enc.submit(sess[i], pt[i]);
  }
  const std::vector<nt::Batcher::Result> ct = enc.flush();
  check(ct.size() == (std::size_t)M, "result count", M);
  // oracle: session s's k-th message has nonce n0[s] + k
  std::vector<std::uint64_t> next(n0);
  bytes want(65535 + 16);
  for (int i = 0; i < M; ++i) {
    const int s = sess[i];
    check(ct[i].session == (std::size_t)s && ct[i].nonce == next[s], "nonce order", i);
    oracle_noise_encrypt(keys[s].data(), next[s]++, nullptr, 0, pt[i].data(), pt[i].size(), want.data());
    check(ct[i].ok && ct[i].msg.size() == pt[i].size() + 16 &&
              std::memcmp(ct[i].msg.data(), want.data(), pt[i].size() + 16) == 0,
          "ciphertext vs oracle", i);
  }
  for (int s = 0; s < S; ++s) check(enc.nonce(s) == next[s], "encrypt nonce advance", s);
  // per-session framed streams, read back in random chunks
  std::vector<bytes> stream(S);
  std::vector<std::vector<int>> order(S);
  for (int i = 0; i < M; ++i) {
    bytes m = ct[i].msg;
    if (i % 97 == 5) m[rng() % m.size()] ^= 0x40;  // tampered
    nt::append_frame(stream[sess[i]], m.data(), m.size());
    order[sess[i]].push_back(i);
  }
  std::vector<int> sub_idx;
  for (int s = 0; s < S; ++s) {
    nt::Deframer df;
    std::size_t off = 0;
    bytes m;
    std::size_t k = 0;
    while (off < stream[s].size()) {
      const std::size_t c = std::min<std::size_t>(1 + rng() % 3000, stream[s].size() - off);
      df.feed(stream[s].data() + off, c);
      off += c;
      while (df.next(m)) {
        dec.submit(s, m);
        sub_idx.push_back(order[s][k++]);
      }
    }
    check(k == order[s].size() && df.buffered() == 0, "deframed all", s);
  }
  const std::vector<nt::Batcher::Result> back = dec.flush();
  check(back.size() == (std::size_t)M, "decrypt count", M);
  for (std::size_t j = 0; j < back.size(); ++j) {
    const int i = sub_idx[j];
    if (i % 97 == 5) {
      check(!back[j].ok, "tampered record rejected", i);
    } else {
      check(back[j].ok && back[j].msg == pt[i], "decrypt round trip", i);
    }
  }
  for (int s = 0; s < S; ++s) check(dec.nonce(s) == next[s], "decrypt nonce advance (failures too)", s);
  // framing limits
  bool threw = false;
  try {
    bytes big(65536), st;
    nt::append_frame(st, big.data(), big.size());
  } catch (const std::length_error &) {
    threw = true;
  }
  check(threw, "frame > 65535 refused", 0);
  // a session without a key (all-zero k, HasKey() false) is refused by both
  // batch objects instead of producing unkeyed "ciphertext" 
  {
    noise::CipherState nokey;
    nokey.initialize_key(std::array<std::uint8_t, 32>{});  // explicitly all zero
    for (int which = 0; which < 2; ++which) {
      threw = false;
      try {
        if (which == 0) {
          nt::Batcher b(nt::Batcher::Direction::Encrypt);
          b.add_session(nokey);
        } else {
          nt::Pipeline::Options po;
          po.depth = 2;
          po.slot_records = 16;
          nt::Pipeline p(nt::Pipeline::Direction::Encrypt, po);
          p.add_session(nokey);
        }
      } catch (const std::invalid_argument &) {
        threw = true;
      }
      check(threw, which ? "pipeline refuses a keyless session" : "batcher refuses a keyless session", which);
    }
  }
  std::printf("sessions %d messages %d: %s (%d failures)\n", S, M, fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
