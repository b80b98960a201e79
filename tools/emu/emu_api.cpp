// emu_api.cpp -- the C ABI's host-buffer entry points (noise_gpu_api.hip)
// with their kernels (the latency kernel single_kernels.hip, the lane walk,
// the records path, the host pipeline) compiled as host C++ through the HIP
// stand-in, under AddressSanitizer, against the C oracle.  After every call
// it scans every buffer the engine allocated (tracked by the stand-in's
// hipMalloc / hipHostMalloc) and requires it to be all zero -- no key,
// plaintext, ciphertext or one-time key left behind in staging or scratch
// (the reference wipes after every use: monocypher.c:163-167,
// noise.cpp:221-223).  The one exception is the 4-byte done word at the head
// of the latency path's mapped staging.
//
//   emu_api            -> "emu_api ok (N calls, M scans)" or FAIL lines
#include <dirent.h>
#include <sanitizer/common_interface_defs.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "noise_gpu.h"
#include "launchers.hpp"

namespace noise_amd {  // single_kernels.hip: emulated asynchronously (below)
void k_aead_resident(uint8_t *req, uint8_t *base, uint32_t last, uint64_t idle_ticks);
extern uint32_t emu_req_check_flip;  // noise_gpu_api.hip (emulation build only)
}

extern "C" {
void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad, size_t ad_len,
                          const uint8_t *pt, size_t len, uint8_t *out);
int oracle_noise_decrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad, size_t ad_len,
                         const uint8_t *ct, size_t ct_len, uint8_t *out);
void oracle_rekey(const uint8_t key[32], uint8_t out[32]);
}

static int fails = 0, scans = 0;
static std::atomic<int> calls{0};
static std::atomic<const char *> phase{"start"};

// Watchdog: a progress line on stderr every 30 s (calls done, phase); after
// 120 s without a finished call it prints every thread's stack (SIGUSR2 to
// each task of the process; the handler prints its own thread's stack with
// the sanitizer's unwinder), once, so a stall names itself instead of
// running into the test's time limit.
// The handler is a last-resort diagnostic (it runs only after a 120-s stall;
// the sanitizer's unwinder is not async-signal-safe).  SA_RESTART: the sleeps,
// futex waits and barrier waits the signal interrupts in the emulated kernel
// threads resume instead of returning early, so the run after a dump behaves
// as the stalled run did.
static void stack_handler(int) { __sanitizer_print_stack_trace(); }
static void dump_all_stacks() {
  struct sigaction sa {};
  sa.sa_handler = stack_handler;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART;
  sigaction(SIGUSR2, &sa, nullptr);
  const pid_t me = (pid_t)syscall(SYS_gettid);
  if (DIR *d = opendir("/proc/self/task")) {
    while (dirent *e = readdir(d)) {
      const pid_t tid = (pid_t)std::atoi(e->d_name);
      if (tid <= 0 || tid == me) continue;
      std::fprintf(stderr, "---- thread %d\n", (int)tid);
      syscall(SYS_tgkill, getpid(), tid, SIGUSR2);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    closedir(d);
  }
}
static void start_watchdog() {
  std::thread([] {
    using namespace std::chrono;
    const auto t0 = steady_clock::now();
    auto last_change = t0;
    int last_calls = -1;
    bool dumped = false;
    for (;;) {
      std::this_thread::sleep_for(seconds(30));
      const auto now = steady_clock::now();
      const int c = calls.load();
      if (c != last_calls) last_calls = c, last_change = now;
      std::fprintf(stderr, "[emu_api watchdog] %.0f s: %d calls, phase %s\n",
                   duration<double>(now - t0).count(), c, phase.load());
      if (!dumped && now - last_change > seconds(120)) {
        dumped = true;
        std::fprintf(stderr, "[emu_api watchdog] no call finished for 120 s: stacks of every thread\n");
        dump_all_stacks();
      }
    }
  }).detach();
}
#define CHECK(c, ...)                      \
  do {                                     \
    if (!(c)) {                            \
      if (fails < 30) {                    \
        std::printf("FAIL: " __VA_ARGS__); \
        std::printf("\n");                 \
      }                                    \
      ++fails;                             \
    }                                      \
  } while (0)

// every engine allocation zero (bytes [0,4) of host allocations: done word;
// resident mode also leaves the alive word [8,12) of the host image and the
// four seq words [16c, 16c + 4) of the request image's request line)
static void scan(const char *after, bool resident = false) {
  ++scans;
  std::lock_guard<std::mutex> lk(emu::alloc_mu);
  for (const auto &[p, a] : emu::allocations()) {
    const uint8_t *b = static_cast<const uint8_t *>(p);
    const bool req = resident && !a.host && a.size == noise_amd::kOneReqBytes;
    for (size_t i = a.host ? 4 : 0; i < a.size; ++i)
      if (b[i] && !(resident && a.host && i >= 8 && i < 12) && !(req && i < 64 && i % 16 < 4)) {
        CHECK(false, "after %s: %s allocation of %zu bytes has byte %zu = %02x", after,
              a.host ? "host" : "device", a.size, i, b[i]);
        break;
      }
  }
}

// each phase's start on stdout with the time since the run began
static const auto g_t0 = std::chrono::steady_clock::now();
static void enter(const char *what) {
  phase = what;
  std::printf("[%7.1f s] %s\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - g_t0).count(), what);
  std::fflush(stdout);
}

static void refused_request(const char *what, double limit_s, const uint8_t key[32], std::mt19937_64 &rng) {
  enter(what);
  std::vector<uint8_t> buf(64 + 16), pt(64), want(64 + 16);
  for (auto &x : pt) x = (uint8_t)rng();
  std::memcpy(buf.data(), pt.data(), 64);
  noise_amd::emu_req_check_flip = 0x00010000u;
  const auto t0 = std::chrono::steady_clock::now();
  ++calls;
  int rc = noise_gpu_encrypt_host(key, 5, nullptr, 0, buf.data(), 64);
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  noise_amd::emu_req_check_flip = 0u;
  CHECK(rc == NOISE_GPU_E_HIP && secs < limit_s, "refused request (%s): rc=%d after %.1f s", what, rc, secs);
  std::printf("refused request (%s): rc %d after %.2f s (%s)\n", what, rc, secs, noise_gpu_last_error());
  scan("refused request", true);
  oracle_noise_encrypt(key, 6, nullptr, 0, pt.data(), 64, want.data());
  std::memcpy(buf.data(), pt.data(), 64);
  ++calls;
  rc = noise_gpu_encrypt_host(key, 6, nullptr, 0, buf.data(), 64);
  CHECK(rc == NOISE_GPU_OK && buf == want, "after the refused request (%s): rc=%d", what, rc);
  scan("after the refused request", true);
}

int main() {
  start_watchdog();
  std::mt19937_64 rng(12345);
  auto rbytes = [&](size_t n) {
    std::vector<uint8_t> v(n);
    for (auto &x : v) x = (uint8_t)rng();
    return v;
  };
  uint8_t key[32];
  for (auto &x : key) x = (uint8_t)rng();
  // ---- single records: latency kernel (AD <= 8192) and the staged path
  enter("single records (launch mode)");
  const size_t lens[] = {0, 1, 15, 16, 17, 63, 64, 65, 100, 1000, 1024, 1040, 4096, 5000, 16384,
                         65519, 65535, 70000};
  const size_t ads[] = {0, 7, 64, 100, 9000};
  for (size_t L : lens)
    for (size_t A : ads) {
      if (L > 20000 && A == 9000) continue;
      const uint64_t n = rng() % 1000 + (L == 16 ? (1ull << 32) - 1 : 0);
      const auto pt = rbytes(L), ad = rbytes(A);
      std::vector<uint8_t> want(L + 16), buf(pt);
      buf.resize(L + 16);
      oracle_noise_encrypt(key, n, ad.data(), A, pt.data(), L, want.data());
      ++calls;
      int rc = noise_gpu_encrypt_host(key, n, A ? ad.data() : nullptr, A, buf.data(), L);
      CHECK(rc == NOISE_GPU_OK && buf == want, "encrypt_host L=%zu A=%zu rc=%d", L, A, rc);
      scan("encrypt_host");
      ++calls;
      rc = noise_gpu_decrypt_host(key, n, A ? ad.data() : nullptr, A, buf.data(), L + 16);
      CHECK(rc == NOISE_GPU_OK && std::memcmp(buf.data(), pt.data(), L) == 0,
            "decrypt_host L=%zu A=%zu rc=%d", L, A, rc);
      scan("decrypt_host");
      // tampered: MAC failure, buffer untouched
      std::vector<uint8_t> bad(want);
      bad[rng() % bad.size()] ^= 0x20;
      const std::vector<uint8_t> snap(bad);
      ++calls;
      rc = noise_gpu_decrypt_host(key, n, A ? ad.data() : nullptr, A, bad.data(), L + 16);
      CHECK(rc == NOISE_GPU_E_MAC && bad == snap, "tampered L=%zu A=%zu rc=%d", L, A, rc);
      scan("decrypt_host (tampered)");
    }
  // ---- single records through the resident latency kernel (opt-in): the
  // emulated launch runs it to its idle exit, so every further request is
  // picked up by a relaunch from the host's wait loop (the lost-doorbell path)
  enter("resident, synchronous instances");
  CHECK(noise_gpu_set_resident(1, 300) == NOISE_GPU_OK, "set_resident on");
  CHECK(noise_gpu_set_resident(1, 20000000) == NOISE_GPU_E_ARG, "idle above 10 s refused");
  for (size_t L : {0ul, 17ul, 1024ul, 4096ul, 65535ul, 70000ul})
    for (size_t A : {0ul, 64ul, 9000ul}) {
      const uint64_t n = rng();
      const auto pt = rbytes(L), ad = rbytes(A);
      std::vector<uint8_t> want(L + 16), buf(pt);
      buf.resize(L + 16);
      oracle_noise_encrypt(key, n, ad.data(), A, pt.data(), L, want.data());
      ++calls;
      int rc = noise_gpu_encrypt_host(key, n, A ? ad.data() : nullptr, A, buf.data(), L);
      CHECK(rc == NOISE_GPU_OK && buf == want, "resident encrypt_host L=%zu A=%zu rc=%d", L, A, rc);
      scan("resident encrypt_host", true);
      ++calls;
      rc = noise_gpu_decrypt_host(key, n, A ? ad.data() : nullptr, A, buf.data(), L + 16);
      CHECK(rc == NOISE_GPU_OK && std::memcmp(buf.data(), pt.data(), L) == 0,
            "resident decrypt_host L=%zu A=%zu rc=%d", L, A, rc);
      scan("resident decrypt_host", true);
      std::vector<uint8_t> bad(want);
      bad[rng() % bad.size()] ^= 0x02;
      const std::vector<uint8_t> snap(bad);
      ++calls;
      rc = noise_gpu_decrypt_host(key, n, A ? ad.data() : nullptr, A, bad.data(), L + 16);
      CHECK(rc == NOISE_GPU_E_MAC && bad == snap, "resident tampered L=%zu A=%zu rc=%d", L, A, rc);
      scan("resident decrypt_host (tampered)", true);
    }
  // consecutive nonces under two interleaved keys: after (key, n) the kernel
  // speculates on (key, n + 1), so from the second record of each run on the
  // speculated path (one_body_fast) answers -- every size class around its
  // limits (63 keystream blocks, 256 Poly1305 blocks), tampering included.
  // The resident kernel runs asynchronously here (as on a GPU: one instance
  // serves many requests) with a long idle time, so its slots survive.
  // a request line no instance takes (its check word corrupted): every
  // relaunched instance sees it whole on its first poll and refuses it, so
  // the host's wait gives up after its relaunch cap -- E_HIP at once, not a
  // loop -- and the next call on the context works
  refused_request("synchronous instances", 15.0, key, rng);
  enter("resident, one asynchronous instance");
  emu::async_kernel = reinterpret_cast<void *>(&noise_amd::k_aead_resident);
  CHECK(noise_gpu_set_resident(1, 5000000) == NOISE_GPU_OK, "set_resident long idle");
  {
    uint8_t key2[32];
    for (auto &x : key2) x = (uint8_t)rng();
    for (size_t L : {0ul, 1ul, 16ul, 17ul, 1000ul, 1024ul, 3952ul, 3953ul, 4032ul, 4033ul, 4096ul})
      for (size_t A : {0ul, 64ul, 100ul}) {
        const uint64_t n0 = rng() >> 1, m0 = rng() >> 1;
        for (int i = 0; i < 3; ++i)
          for (int which = 0; which < 2; ++which) {
            const uint8_t *k = which ? key2 : key;
            const uint64_t n = (which ? m0 : n0) + (uint64_t)i;
            const auto pt = rbytes(L), ad = rbytes(A);
            std::vector<uint8_t> want(L + 16), buf(pt);
            buf.resize(L + 16);
            oracle_noise_encrypt(k, n, ad.data(), A, pt.data(), L, want.data());
            ++calls;
            int rc = noise_gpu_encrypt_host(k, n, A ? ad.data() : nullptr, A, buf.data(), L);
            CHECK(rc == NOISE_GPU_OK && buf == want, "resident run encrypt L=%zu A=%zu i=%d rc=%d", L,
                  A, i, rc);
            scan("resident run encrypt", true);
            // the same record decrypted at n + 1's turn: the slot now holds n + 1
            if (i == 1) {
              std::vector<uint8_t> bad(want);
              bad[rng() % bad.size()] ^= 0x10;
              const std::vector<uint8_t> snap(bad);
              ++calls;
              rc = noise_gpu_decrypt_host(k, n + 1, A ? ad.data() : nullptr, A, bad.data(), L + 16);
              CHECK(rc == NOISE_GPU_E_MAC && bad == snap, "resident run wrong nonce L=%zu rc=%d", L, rc);
              scan("resident run wrong nonce", true);
            }
          }
        // decrypt a run: n0 misses, n0 + 1 and n0 + 2 hit (the second one tampered)
        for (int i = 0; i < 3; ++i) {
          const uint64_t n = n0 + (uint64_t)i;
          const auto pt = rbytes(L), ad = rbytes(A);
          std::vector<uint8_t> ct(L + 16);
          oracle_noise_encrypt(key, n, ad.data(), A, pt.data(), L, ct.data());
          if (i == 2) ct[rng() % ct.size()] ^= 0x40;
          std::vector<uint8_t> buf(ct);
          ++calls;
          const int rc = noise_gpu_decrypt_host(key, n, A ? ad.data() : nullptr, A, buf.data(), L + 16);
          if (i == 2)
            CHECK(rc == NOISE_GPU_E_MAC && buf == ct, "resident run tampered L=%zu rc=%d", L, rc);
          else
            CHECK(rc == NOISE_GPU_OK && std::memcmp(buf.data(), pt.data(), L) == 0,
                  "resident run decrypt L=%zu A=%zu i=%d rc=%d", L, A, i, rc);
          scan("resident run decrypt", true);
        }
      }
  }
  // the same with one long-lived instance that keeps polling: the host's
  // wait runs into its 10-s limit, stops the instance (bounded) and fails
  // the call; the next call relaunches and works
  refused_request("asynchronous instance", 15.0, key, rng);
  CHECK(noise_gpu_set_resident(0, 0) == NOISE_GPU_OK, "set_resident off");
  enter("rekey, batches, contexts");
  emu::async_kernel = nullptr;
  // ---- rekey
  for (int i = 0; i < 4; ++i) {
    uint8_t k[32], w[32];
    for (auto &x : k) x = (uint8_t)(i ? rng() : 0);
    oracle_rekey(k, w);
    ++calls;
    const int rc = noise_gpu_rekey_host(k);
    CHECK(rc == NOISE_GPU_OK && std::memcmp(k, w, 32) == 0, "rekey_host %d", i);
    scan("rekey_host");
  }
  // ---- descriptor batch between host buffers (records path + its scratch)
  for (int big = 0; big < 2; ++big) {
    const uint32_t nrec = big ? 2300 : 40;  // above / below the classifier threshold
    const uint32_t nkeys = 3;
    const auto keys = rbytes(32 * nkeys);
    std::vector<noise_gpu_record> recs(nrec);
    std::vector<std::vector<uint8_t>> pts(nrec);
    uint64_t in_b = 0, out_b = 0;
    for (uint32_t i = 0; i < nrec; ++i) {
      const uint32_t L = (i % 13 == 0) ? 2048 + (uint32_t)(rng() % 5000) : (uint32_t)(rng() % 700);
      pts[i] = rbytes(L);
      recs[i] = noise_gpu_record{in_b, out_b, rng() % 100000, 0, L, 0, (uint32_t)(rng() % nkeys), 0};
      in_b += (L + 15) & ~15u;
      out_b += (L + 31) & ~15u;
    }
    std::vector<uint8_t> hin(in_b + 1), hout(out_b + 1);
    for (uint32_t i = 0; i < nrec; ++i)
      if (!pts[i].empty()) std::memcpy(hin.data() + recs[i].in_off, pts[i].data(), pts[i].size());
    ++calls;
    int rc = noise_gpu_encrypt_records_host(keys.data(), nkeys, recs.data(), nrec, hin.data(), in_b,
                                            hout.data(), out_b, nullptr, 0);
    CHECK(rc == NOISE_GPU_OK, "encrypt_records_host rc=%d", rc);
    std::vector<uint8_t> w(8192);
    for (uint32_t i = 0; i < nrec; ++i) {
      oracle_noise_encrypt(keys.data() + 32 * recs[i].key_idx, recs[i].nonce, nullptr, 0,
                           pts[i].data(), pts[i].size(), w.data());
      CHECK(std::memcmp(hout.data() + recs[i].out_off, w.data(), pts[i].size() + 16) == 0,
            "records_host record %u (len %u)", i, recs[i].len);
    }
    scan(big ? "encrypt_records_host (classified)" : "encrypt_records_host (small)");
  }
  // ---- uniform batch between host buffers (pipeline; the tile kernel's
  // wire-order gather below 1 KiB, the record-wise one from 1 KiB), at
  // every length the tile kernel serves: G = 1 .. 64 lanes per record
  for (uint32_t L : {64u, 128u, 192u, 256u, 512u, 1024u, 2048u, 4096u, 8192u, 16384u}) {
    const uint32_t R = L >= 4096 ? 70 : 300;
    const auto pt = rbytes((size_t)L * R);
    std::vector<uint8_t> ct((size_t)(L + 16) * R), back((size_t)L * R), st(R, 9);
    double secs = 0;
    ++calls;
    int rc = noise_gpu_encrypt_uniform_host(key, 7, pt.data(), L, ct.data(), L + 16, L, R, &secs);
    CHECK(rc == NOISE_GPU_OK, "encrypt_uniform_host rc=%d", rc);
    std::vector<uint8_t> w(L + 16);
    for (uint32_t i = 0; i < R; ++i) {
      oracle_noise_encrypt(key, 7 + i, nullptr, 0, pt.data() + (size_t)i * L, L, w.data());
      CHECK(std::memcmp(ct.data() + (size_t)i * (L + 16), w.data(), L + 16) == 0, "uniform_host %u", i);
    }
    scan("encrypt_uniform_host");
    ++calls;
    rc = noise_gpu_decrypt_uniform_host(key, 7, ct.data(), L + 16, back.data(), L, L, st.data(), R,
                                        &secs);
    CHECK(rc == NOISE_GPU_OK && back == pt, "decrypt_uniform_host rc=%d", rc);
    for (uint32_t i = 0; i < R; ++i) CHECK(st[i] == 0, "uniform_host status %u", i);
    scan("decrypt_uniform_host");
  }
  // ---- explicit device context: same results through its own staging
  {
    const size_t live0 = emu::allocations().size();  // the thread's own contexts
    noise_gpu_ctx *ctx = nullptr;
    CHECK(noise_gpu_ctx_create(0, &ctx) == NOISE_GPU_OK && ctx, "ctx_create");
    CHECK(noise_gpu_ctx_destroy(ctx) == NOISE_GPU_OK, "ctx_destroy");
    CHECK(noise_gpu_ctx_create(5, &ctx) == NOISE_GPU_E_ARG, "ctx_create bad index");
    CHECK(noise_gpu_ctx_create(0, &ctx) == NOISE_GPU_OK && ctx, "ctx_create again");
    int dev = -1;
    CHECK(noise_gpu_ctx_device(ctx, &dev) == NOISE_GPU_OK && dev == 0, "ctx_device");
    CHECK(noise_gpu_ctx_set_resident(ctx, 1, 200) == NOISE_GPU_OK, "ctx resident on");
    for (size_t L : {0, 17, 1024, 70000}) {
      const auto pt = rbytes(L), ad = rbytes(64);
      std::vector<uint8_t> want(L + 16), buf(pt);
      buf.resize(L + 16);
      oracle_noise_encrypt(key, 99, ad.data(), 64, pt.data(), L, want.data());
      ++calls;
      int rc = noise_gpu_ctx_encrypt_host(ctx, key, 99, ad.data(), 64, buf.data(), L);
      CHECK(rc == NOISE_GPU_OK && buf == want, "ctx encrypt_host L=%zu rc=%d", L, rc);
      scan("ctx encrypt_host", true);
      ++calls;
      rc = noise_gpu_ctx_decrypt_host(ctx, key, 99, ad.data(), 64, buf.data(), L + 16);
      CHECK(rc == NOISE_GPU_OK && std::memcmp(buf.data(), pt.data(), L) == 0,
            "ctx decrypt_host L=%zu rc=%d", L, rc);
      scan("ctx decrypt_host", true);
    }
    {
      const uint32_t L = 1024, R = 100;
      const auto pt = rbytes((size_t)L * R);
      std::vector<uint8_t> ct((size_t)(L + 16) * R), back((size_t)L * R), st(R, 9);
      double secs = 0;
      ++calls;
      int rc = noise_gpu_ctx_encrypt_uniform_host(ctx, key, 3, pt.data(), L, ct.data(), L + 16, L,
                                                  R, &secs);
      std::vector<uint8_t> w(L + 16);
      oracle_noise_encrypt(key, 3 + R - 1, nullptr, 0, pt.data() + (size_t)(R - 1) * L, L, w.data());
      CHECK(rc == NOISE_GPU_OK &&
                std::memcmp(ct.data() + (size_t)(R - 1) * (L + 16), w.data(), L + 16) == 0,
            "ctx encrypt_uniform_host rc=%d", rc);
      scan("ctx encrypt_uniform_host", true);
      ++calls;
      rc = noise_gpu_ctx_decrypt_uniform_host(ctx, key, 3, ct.data(), L + 16, back.data(), L, L,
                                              st.data(), R, &secs);
      CHECK(rc == NOISE_GPU_OK && back == pt, "ctx decrypt_uniform_host rc=%d", rc);
      scan("ctx decrypt_uniform_host", true);
    }
    {  // a classified descriptor batch: records scratch + companion stream on the ctx's stream
      const uint32_t nrec = 300, L = 2100;
      const auto pt = rbytes((size_t)nrec * 2112);
      std::vector<noise_gpu_record> recs(nrec);
      for (uint32_t i = 0; i < nrec; ++i)
        recs[i] = noise_gpu_record{2112ull * i, 2128ull * i, i, 0, L, 0, 0, 0};
      std::vector<uint8_t> out((size_t)nrec * 2128);
      ++calls;
      const int rc = noise_gpu_ctx_encrypt_records_host(ctx, key, 1, recs.data(), nrec, pt.data(),
                                                        pt.size(), out.data(), out.size(), nullptr, 0);
      std::vector<uint8_t> w(L + 16);
      oracle_noise_encrypt(key, nrec - 1, nullptr, 0, pt.data() + 2112ull * (nrec - 1), L, w.data());
      CHECK(rc == NOISE_GPU_OK && std::memcmp(out.data() + 2128ull * (nrec - 1), w.data(), L + 16) == 0,
            "ctx encrypt_records_host rc=%d", rc);
      scan("ctx encrypt_records_host", true);
    }
    CHECK(noise_gpu_ctx_destroy(ctx) == NOISE_GPU_OK, "ctx_destroy");
    // destroy freed everything the context allocated, records scratch included
    CHECK(emu::allocations().size() == live0, "ctx_destroy left %zu allocations",
          emu::allocations().size() - live0);
    CHECK(noise_gpu_ctx_encrypt_host(nullptr, key, 0, nullptr, 0, nullptr, 0) == NOISE_GPU_E_ARG,
          "null ctx");
  }
  // the documented maximum of the host uniform pipeline is refused above it
  {
    std::vector<uint8_t> a(64), b(64);
    double secs = 0;
    CHECK(noise_gpu_encrypt_uniform_host(key, 0, a.data(), NOISE_GPU_UNIFORM_HOST_MAX_LEN + 16, b.data(),
                                         NOISE_GPU_UNIFORM_HOST_MAX_LEN + 32,
                                         NOISE_GPU_UNIFORM_HOST_MAX_LEN + 16, 1, &secs) == NOISE_GPU_E_ARG,
          "uniform_host above the maximum length");
  }
  // every per-thread context released: nothing the engine allocated is left
  CHECK(noise_gpu_thread_release() == NOISE_GPU_OK, "thread_release");
  CHECK(emu::allocations().empty(), "thread_release left %zu allocations", emu::allocations().size());
  if (fails) {
    std::printf("emu_api FAIL (%d failures, %d calls, %d scans)\n", fails, calls.load(), scans);
    return 1;
  }
  std::printf("emu_api ok (%d calls, %d scans)\n", calls.load(), scans);
  return 0;
}
