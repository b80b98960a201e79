// noise_gpu_api.hip -- the C ABI (include/noise_gpu.h) over the gfx950
// kernels.  Argument checks, launches, and the host-buffer entry points
// (pinned staging for single records; chunked, multi-stream pipelines for
// host-resident batches).  Nothing here computes ChaCha20 or Poly1305:
// every record goes through the HIP kernels, and without a gfx950 device
// every entry point fails with NOISE_GPU_E_NODEV / NOISE_GPU_E_HIP.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <vector>
#include <cstring>
#include <new>
#include <string>

#include "launchers.hpp"
#include "noise_amd/dev_mem.hpp"
#include "noise_gpu.h"

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char *what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return NOISE_GPU_E_HIP;
}

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

// Is a gfx950 device current?  Cached per thread and device.
int check_device() {
  // per thread: the device last checked and its verdict -- the single-record
  // path calls this per record, so a known device costs one hipGetDevice
  thread_local int cached_dev = -1, cached_ok = 0;
  int dev = 0;
  if (cached_dev >= 0 && hipGetDevice(&dev) == hipSuccess && dev == cached_dev)
    return cached_ok ? NOISE_GPU_OK : NOISE_GPU_E_NODEV;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    g_last_error = "no HIP device visible";
    return NOISE_GPU_E_NODEV;
  }
  HIP_TRY(hipGetDevice(&dev));
  if (dev == cached_dev) return cached_ok ? NOISE_GPU_OK : NOISE_GPU_E_NODEV;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  cached_dev = dev;
  cached_ok = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
  if (!cached_ok) {
    g_last_error = std::string("device is ") + prop.gcnArchName +
                   ", this engine is built for gfx950 only";
    return NOISE_GPU_E_NODEV;
  }
  return NOISE_GPU_OK;
}

void key_words(const uint8_t *key, uint32_t w[8]) { std::memcpy(w, key, 32); }

// An all-zero key is "no key" (Noise HasKey() false; CipherState never
// calls the engine then): refused rather than used as a public key.
bool key_absent(const uint8_t *key) {
  uint8_t acc = 0;
  for (int i = 0; i < 32; ++i) acc |= key[i];
  return acc == 0;
}

int arg_fail(const char *msg) {
  g_last_error = msg;
  return NOISE_GPU_E_ARG;
}

// Validate a uniform batch.  enc: in = len-byte records, out = len+16.
int check_uniform(bool decrypt, const void *in, uint64_t in_stride,
                  const void *out, uint64_t out_stride, uint32_t len,
                  const void *ad, uint32_t ad_len, const void *status,
                  uint64_t nrec) {
  if (nrec == 0) return NOISE_GPU_OK;
  const uint64_t in_rec = decrypt ? (uint64_t)len + 16 : len;
  const uint64_t out_rec = decrypt ? len : (uint64_t)len + 16;
  if (!in || !out) return arg_fail("null record buffer");
  if ((nrec > 1 && in_stride < in_rec) || (nrec > 1 && out_stride < out_rec))
    return arg_fail("record stride smaller than the record");
  if (in == out && in_stride != out_stride)
    return arg_fail("in-place batches need equal strides");
  if (in == out && nrec > 1 && in_stride < (uint64_t)len + 16)
    return arg_fail("in-place stride must hold len+16 bytes");
  if (ad_len && !ad) return arg_fail("ad_len > 0 with null ad");
  if (decrypt && !status) return arg_fail("null status buffer");
  return NOISE_GPU_OK;
}

// Per-thread staging for the synchronous host-buffer entry points.
struct Staging {
  int dev = -1;
  hipStream_t stream = nullptr;
  uint8_t *d = nullptr, *h = nullptr;
  size_t cap = 0;
  ~Staging() { release(); }
  // free everything, including the records scratch and companion stream the
  // descriptor path cached for this staging stream (records_scratch_release)
  void release() {
    int cur = -1;
    if (stream && dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
    if (stream) (void)noise_amd::records_scratch_release(stream);
    if (d) {  // wiped and freed stream-ordered (dev_mem.hpp), then waited for
      (void)noise_amd::dev_wipe_free(d, cap, stream);
      (void)hipStreamSynchronize(stream);
    }
    if (h) {
      std::memset(h, 0, cap);
      (void)hipHostFree(h);
    }
    if (stream) (void)hipStreamDestroy(stream);
    if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
    d = h = nullptr;
    stream = nullptr;
    cap = 0;
    dev = -1;
  }
  // hygiene after a call: the pinned image and the device scratch
  // (hipMemsetAsync on the staging stream; a later call's copies queue after it)
  void wipe(size_t bytes) {
    if (bytes > cap) bytes = cap;
    if (h) std::memset(h, 0, bytes);
    if (d && stream) (void)hipMemsetAsync(d, 0, bytes, stream);
  }
  int reserve(size_t bytes) {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != dev) {  // device switched: drop the old device's resources
      release();
      dev = cur;
      HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }
    if (bytes <= cap) return NOISE_GPU_OK;
    size_t want = cap ? cap : 4096;
    while (want < bytes) want *= 2;
    // grow: the old device buffer is wiped and freed after this stream's
    // earlier work (a hipFree would wait for every stream of the device)
    if (d) (void)noise_amd::dev_wipe_free(d, cap, stream);
    if (h) {
      (void)hipStreamSynchronize(stream);  // its copies are done with it
      std::memset(h, 0, cap);
      (void)hipHostFree(h);
    }
    d = nullptr; h = nullptr; cap = 0;
    HIP_TRY(noise_amd::dev_alloc(reinterpret_cast<void **>(&d), want, stream));
    HIP_TRY(hipHostMalloc(&h, want, hipHostMallocDefault));
    cap = want;
    return NOISE_GPU_OK;
  }
};
// Contexts are kept per (thread, device): a thread that serves several GPUs
// (hipSetDevice between calls) keeps every device's streams and buffers
// instead of freeing and re-creating them on each switch.  Devices beyond
// kMaxCtxDev share slots, whose reserve() re-targets on a switch.
constexpr int kMaxCtxDev = 16;
template <class Ctx>
static Ctx *ctx_of(Ctx (&tab)[kMaxCtxDev]) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  return &tab[dev % kMaxCtxDev];
}
thread_local Staging g_stage_tab[kMaxCtxDev];
// An explicit noise_gpu_ctx (noise_gpu_ctx_* entry points) substitutes its
// own contexts for the thread's for the duration of one call.
thread_local Staging *tl_stage = nullptr;
// the calling thread's staging on its current device (nullptr: no device)
#define NOISE_STAGE(var)                                                       \
  Staging *var##_p = tl_stage ? tl_stage : ctx_of(g_stage_tab);                \
  if (!var##_p) return hip_fail(hipErrorInvalidDevice, "hipGetDevice");             \
  Staging &var = *var##_p

// Per-thread latency-path context (single_kernels.hip): a stream and a
// host-mapped, coherent pinned staging image the kernel reads and writes
// over PCIe; completion is a done word the kernel stores last.  In resident
// mode (noise_gpu_set_resident) one workgroup stays on the GPU and serves
// requests rung through the image's request line instead of one launch per
// record; it leaves on its own after idle_us without requests (and is
// relaunched by the next one), on the stop word, and at teardown.
constexpr uint32_t kResidentIdleDefaultUs = 20000;
constexpr std::chrono::seconds kOneWaitLimit{10};
// fresh instances launched for one request that all left without taking it
// (each sees the complete request on its first poll) before the call fails
constexpr uint32_t kResidentMaxRelaunch = 8;
constexpr uint32_t kResidentIdleMaxUs = 10000000;
struct OneCtx;
// contexts whose resident kernel may be running (stopped at library unload;
// never destroyed, so the unload hook can still read them)
std::mutex &resident_mu() {
  static std::mutex *m = new std::mutex;
  return *m;
}
std::vector<OneCtx *> &resident_list() {
  static std::vector<OneCtx *> *v = new std::vector<OneCtx *>;
  return *v;
}
void resident_track(OneCtx *c, bool on);
}  // namespace
#if defined(NOISE_HIP_EMU)
namespace noise_amd {
uint32_t emu_req_check_flip = 0;  // tools/emu/emu_api.cpp: corrupts the next request's check word
}
#endif
namespace {
constexpr uint32_t kOneAliveOff = 8;  // u32 in the done line: 1 while an instance runs

// Where the resident kernel's request image lives (NOISE_GPU_RESIDENT_REQ,
// read when the image is allocated): "fine" (default: fine-grained device
// memory, which the host writes through the PCIe BAR and which stays
// coherent with those writes -- the GPU polls local memory), or "host"
// (host-mapped pinned memory: the GPU polls over PCIe; also the fallback when
// fine-grained device memory cannot be allocated).  Coarse-grained device
// memory (plain hipMalloc) is NOT an option: its lines stay valid in the
// GPU's L2 (zeroed there by hipMemset, or left by an earlier kernel) and
// polls served from L2 never see the host's BAR writes.
enum ReqKind : int { kReqFine = 1, kReqHost = 2 };
static int req_kind_env() {
  const char *e = std::getenv("NOISE_GPU_RESIDENT_REQ");
  return e && !std::strcmp(e, "host") ? kReqHost : kReqFine;
}

struct OneCtx {
  int dev = -1;
  hipStream_t stream = nullptr;
  uint8_t *h = nullptr;  // host view
  uint8_t *d = nullptr;  // device view of the same memory
  size_t cap = 0;
  uint32_t seq = 0;
  bool resident = false;   // opt-in (noise_gpu_set_resident)
  uint32_t idle_us = kResidentIdleDefaultUs;
  bool launched = false;   // a resident instance was launched and may still run
  // resident request image (OneReq, launchers.hpp): host and device views
  uint8_t *hreq = nullptr, *dreq = nullptr;
  int req_kind = kReqFine;
  // The resident instance's stream, on a hardware queue of its own.  The HIP
  // runtime maps a process's streams onto GPU_MAX_HW_QUEUES (4 by default)
  // hardware queues per priority level, and a queue runs its packets in
  // order: a stream sharing the instance's queue -- another thread's batch
  // work, a Pipeline slot -- would wait until the instance idles out (seen on
  // MI355X: a Pipeline slot stuck for the whole resident run).  So the
  // instance runs on a non-blocking stream of the HIGHEST priority, whose
  // queue pool is separate from the normal-priority streams'; it shares a
  // queue only if the process creates more high-priority streams than that
  // pool has queues.  (A CU-masked stream also gets a queue of its own, but
  // it is a blocking stream: every null-stream operation -- hipMemcpy, the
  // stream-ordered allocator -- then waits for the instance.)  `stream` stays
  // the launch path's.
  hipStream_t rstream = nullptr;
  ~OneCtx() { release(); }
  noise_amd::OneRing *ring() { return reinterpret_cast<noise_amd::OneRing *>(h + noise_amd::kOneRingOff); }
  // the instance did not leave on the stop word within kOneWaitLimit: its
  // stream is never synchronised again (that wait would not end) and every
  // later call on this context fails with NOISE_GPU_E_HIP
  bool wedged = false;
  // stop word -> the instance leaves at its next poll (every 32 polls, a few
  // microseconds); wait for its alive word, bounded, before the stream sync
  int stop_resident() {
    if (wedged) {
      g_last_error = "resident latency kernel did not stop (context unusable)";
      return NOISE_GPU_E_HIP;
    }
    if (!launched) return NOISE_GPU_OK;
    volatile uint32_t *stop = &ring()->stop;
    *stop = 1u;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1; *alive() != 0u; ++spin) {
      // an instance that never ran (or faulted) does not clear the word:
      // a stream that has ended or failed needs no more waiting
      if ((spin & 4095u) == 0u && rstream && hipStreamQuery(rstream) != hipErrorNotReady) break;
      if (std::chrono::steady_clock::now() - t0 > kOneWaitLimit) {
        wedged = true;  // the stop word stays set
        g_last_error = "resident latency kernel did not stop within 10 s (context unusable)";
        return NOISE_GPU_E_HIP;
      }
      _mm_pause();
    }
    if (rstream) (void)hipStreamSynchronize(rstream);
    *stop = 0u;
    launched = false;
    resident_track(this, false);
    return NOISE_GPU_OK;
  }
  void release_req() {
    if (!hreq) return;
    if (req_kind == kReqHost) {
      std::memset(hreq, 0, noise_amd::kOneReqBytes);
      (void)hipHostFree(hreq);
    } else {
      (void)hipMemset(dreq, 0, noise_amd::kOneReqBytes);
      (void)hipFree(dreq);
    }
    hreq = dreq = nullptr;
  }
  // the request image, zeroed (the running instance, if any, must be stopped)
  int reserve_req() {
    if (hreq) return NOISE_GPU_OK;
    req_kind = req_kind_env();
    void *p = nullptr;
    if (req_kind == kReqFine &&
               hipExtMallocWithFlags(&p, noise_amd::kOneReqBytes, hipDeviceMallocFinegrained) ==
                   hipSuccess) {
      hreq = dreq = static_cast<uint8_t *>(p);
    } else {
      req_kind = kReqHost;
      HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&hreq), noise_amd::kOneReqBytes,
                            hipHostMallocMapped | hipHostMallocCoherent));
      HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&dreq), hreq, 0));
    }
    HIP_TRY(hipMemset(dreq, 0, noise_amd::kOneReqBytes));
    return NOISE_GPU_OK;
  }
  void release() {
    int cur = -1;
    if (stream && dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
    if (stop_resident() != NOISE_GPU_OK) {
      // a wedged instance still runs from this context's memory: leave it all
      // allocated (leaked) rather than free it under the kernel or hang here
      if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
      return;
    }
    if (stream) (void)hipStreamSynchronize(stream);
    release_req();
    if (rstream) {
      (void)hipStreamSynchronize(rstream);
      (void)hipStreamDestroy(rstream);
      rstream = nullptr;
    }
    if (h) {
      std::memset(h, 0, cap);
      (void)hipHostFree(h);
    }
    if (stream) (void)hipStreamDestroy(stream);
    if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
    h = d = nullptr;
    stream = nullptr;
    cap = 0;
    dev = -1;
    seq = 0;
  }
  int reserve(size_t bytes) {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != dev) {
      release();
      dev = cur;
      HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }
    if (wedged) return stop_resident();
    if (bytes <= cap) return NOISE_GPU_OK;
    // a running instance holds the old image's address
    if (int rc = stop_resident()) return rc;
    size_t want = cap ? cap : 16384;
    while (want < bytes) want *= 2;
    if (h) {
      std::memset(h, 0, cap);
      (void)hipHostFree(h);
    }
    h = d = nullptr;
    cap = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h), want,
                          hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, want);
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0));
    cap = want;
    seq = 0;  // a fresh image: doorbell and done word are 0
    return NOISE_GPU_OK;
  }
  volatile uint32_t *alive() { return reinterpret_cast<volatile uint32_t *>(h + kOneAliveOff); }
  int make_rstream() {
    if (rstream) return NOISE_GPU_OK;
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&rstream, hipStreamNonBlocking, greatest));
    return NOISE_GPU_OK;
  }
  int launch_resident(uint32_t last) {
    if (int rc = make_rstream()) return rc;
    *alive() = 1u;  // the instance clears it when it leaves
    const hipError_t e = noise_amd::launch_aead_resident(dreq, d, last, idle_us, rstream);
    if (e != hipSuccess) return hip_fail(e, "launch_aead_resident");
    if (!launched) resident_track(this, true);
    launched = true;
    return NOISE_GPU_OK;
  }
  // launch already issued (or request rung) with `s`: wait for the done word.
  // A record takes microseconds; no answer within kOneWaitLimit means the
  // kernel cannot see the request (or is wedged): stop it and fail the call
  // rather than spin for ever.
  // by_resident: the request went to the resident instance (else a launch on
  // `stream`, the launch path's)
  //
  // Every 64th spin checks the time limit FIRST, before anything that can
  // `continue` the loop: the wait is bounded whatever the instance does.
  // (Round 4 checked it only on spins = 1023 mod 1024, after the relaunch
  // branch, which fires on spins = 63 mod 64 -- a superset: with the alive
  // word 0 at each of those spins, e.g. an instance that leaves without
  // taking the request, the limit was never reached.)  An instance that left
  // (alive word 0) is relaunched; a request that kResidentMaxRelaunch fresh
  // instances in a row did not take -- each one saw the complete request on
  // its first poll, so the request itself is refused (a torn or corrupted
  // request line: check word or seq) -- fails the call.  No instance runs
  // then, so the context stays usable; one_record wipes the request image.
  int wait(uint32_t s, bool by_resident) {
    hipStream_t wst = by_resident ? rstream : stream;
    volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(h);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t relaunches = 0;
    for (uint64_t spin = 0;; ++spin) {
      if (*done == s) return NOISE_GPU_OK;
      if ((spin & 63u) != 63u) continue;
      const auto waited = std::chrono::steady_clock::now() - t0;
      if (waited > kOneWaitLimit) {
        if (*done == s) return NOISE_GPU_OK;
        if (by_resident) (void)stop_resident();  // bounded; marks the context wedged if it must
        if (!wedged) g_last_error = "latency kernel gave no answer within 10 s";
        return NOISE_GPU_E_HIP;
      }
      // the instance left on its idle timer after its last poll (it clears
      // the alive word last, after any done word it wrote): relaunch now
      // instead of after the first stream query below
      if (by_resident && *alive() == 0u) {
        if (*done == s) return NOISE_GPU_OK;
        if (++relaunches > kResidentMaxRelaunch) {
          g_last_error = "resident latency kernel did not take the request (relaunched without progress)";
          return NOISE_GPU_E_HIP;
        }
        const int rc = launch_resident(s - 1u);
        if (rc) return rc;
        continue;
      }
      // now and then: has the stream failed or ended?  A record takes
      // microseconds: the stream query (a runtime call of ~1 us) is for the
      // rare stall, not for every call's last spins
      if ((spin & 1023u) != 1023u || waited < std::chrono::microseconds(100)) continue;
      const hipError_t e = hipStreamQuery(wst);
      if (e == hipSuccess) {
        if (*done == s) return NOISE_GPU_OK;
        // idled out: its alive word is 0, relaunched above
        if (by_resident && launched && *alive() == 0u) continue;
        g_last_error = "latency kernel ended without its done word";
        return NOISE_GPU_E_HIP;
      }
      if (e != hipErrorNotReady) return hip_fail(e, "latency kernel");
    }
  }
};
thread_local OneCtx g_one_tab[kMaxCtxDev];
thread_local OneCtx *tl_one = nullptr;

void resident_track(OneCtx *c, bool on) {
  std::lock_guard<std::mutex> lk(resident_mu());
  std::vector<OneCtx *> &l = resident_list();
  auto it = std::find(l.begin(), l.end(), c);
  if (on && it == l.end()) l.push_back(c);
  if (!on && it != l.end()) l.erase(it);
}

// Library unload (dlclose, or process exit after the threads' own teardown
// stopped theirs): no resident kernel may outlive the code object it runs
// from.  No HIP calls here (the runtime may already be gone at exit): set
// every stop word, then wait -- bounded -- for each instance's alive word.
__attribute__((destructor)) void resident_stop_all() {
  std::vector<OneCtx *> v;
  {
    std::lock_guard<std::mutex> lk(resident_mu());
    v = resident_list();
  }
  for (OneCtx *c : v) {
    volatile uint32_t *stop = &c->ring()->stop;
    *stop = 1u;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (OneCtx *c : v)
    while (*c->alive() != 0u &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(500)) {
    }
}

// One record through the latency kernel (or the resident one).  dec: in = ct
// (len bytes) + tag.  Returns the kernel's status in *st (decrypt); out
// receives len (+16 on encrypt) bytes.  Staging is wiped after use.
int one_record(bool dec, const uint8_t key[32], uint64_t nonce, const uint8_t *ad, uint32_t ad_len,
               const uint8_t *in, uint32_t len, const uint8_t *tag, uint8_t *out, uint32_t *st) {
  const noise_amd::OneLayout lay = noise_amd::one_layout(ad_len, len);
  OneCtx *cp = tl_one ? tl_one : ctx_of(g_one_tab);
  if (!cp) return hip_fail(hipErrorInvalidDevice, "hipGetDevice");
  OneCtx &c = *cp;
  // resident: the image is sized for the largest request once (the running
  // instance holds its address)
  int rc = c.reserve(c.resident ? noise_amd::one_layout(noise_amd::kOneMaxAd, 65535u).total
                                : lay.total);
  if (rc) return rc;
  if (c.resident && (rc = c.reserve_req())) return rc;
  // the resident kernel serves records of <= 63 keystream blocks; a bigger
  // one is a launch on the launch path's stream (the instance has its own)
  const bool res = c.resident && len <= noise_amd::kResidentMaxLen;
  uint32_t s = ++c.seq;
  if (s == 0) s = c.seq = 1;
  const uint32_t n_inl = res ? noise_amd::req_inline_chunks(ad_len, len, dec) : 0u;
  if (n_inl) {
    // a small record goes inline: its staged image (AD | pad | record | pad
    // | tag) 12 bytes per 16-byte chunk {seq, 3 words} (launchers.hpp OneReq)
    alignas(16) uint8_t im[noise_amd::kReqInlineBytes + 12];
    const uint32_t na16 = (ad_len + 15u) & ~15u, nl16 = (len + 15u) & ~15u;
    std::memset(im, 0, 12u * n_inl);
    if (ad_len) std::memcpy(im, ad, ad_len);
    if (len) std::memcpy(im + na16, in, len);
    if (dec) std::memcpy(im + na16 + nl16, tag, 16);
    __m128i *q = reinterpret_cast<__m128i *>(c.hreq) + 4;
    for (uint32_t i = 0; i < n_inl; ++i) {
      uint32_t w[3];
      std::memcpy(w, im + 12u * i, 12);
      const uint32_t x = s ^ noise_amd::req_chunk_tag(4u + i, w[0], w[1], w[2]);
      _mm_store_si128(q + i, _mm_setr_epi32((int)x, (int)w[0], (int)w[1], (int)w[2]));
      w[0] = w[1] = w[2] = 0u;
    }
    explicit_bzero(im, 12u * n_inl);  // the plaintext copy on the stack goes too
  } else {
    // staged in place: the launch path's host image, or the resident
    // request image's DMA area
    uint8_t *img = res ? c.hreq + noise_amd::kReqStageOff : c.h;
    if (ad_len) std::memcpy(img + lay.ad, ad, ad_len);
    if (len) std::memcpy(img + lay.in, in, len);
    if (dec) std::memcpy(img + lay.tag, tag, 16);
  }
  uint32_t k[8];
  key_words(key, k);
  if (res) {
    // the request line: four 16-byte chunks, each {seq ^ its tag, 3 payload
    // words} (launchers.hpp req_chunk_tag), stored whole (16-byte aligned SSE
    // stores) after an sfence that orders them behind the staged bytes
    // (write-combined device memory); the GPU takes the request once all four
    // (and any inline chunks) decode to the new seq
    _mm_sfence();
    const uint32_t meta = len | (ad_len << 16) | ((uint32_t)dec << 30);
    const uint32_t nlo = (uint32_t)nonce, nhi = (uint32_t)(nonce >> 32);
    uint32_t x3 = s ^ noise_amd::req_chunk_tag(3u, k[6], k[7], 0u);
#if defined(NOISE_HIP_EMU)
    x3 ^= noise_amd::emu_req_check_flip;  // tools/emu only: a request line the instance must refuse
#endif
    __m128i *q = reinterpret_cast<__m128i *>(c.hreq);
    _mm_store_si128(q + 1, _mm_setr_epi32((int)(s ^ noise_amd::req_chunk_tag(1u, k[0], k[1], k[2])), (int)k[0],
                                          (int)k[1], (int)k[2]));
    _mm_store_si128(q + 2, _mm_setr_epi32((int)(s ^ noise_amd::req_chunk_tag(2u, k[3], k[4], k[5])), (int)k[3],
                                          (int)k[4], (int)k[5]));
    _mm_store_si128(q + 3, _mm_setr_epi32((int)x3, (int)k[6], (int)k[7], 0));
    _mm_store_si128(q + 0, _mm_setr_epi32((int)(s ^ noise_amd::req_chunk_tag(0u, meta, nlo, nhi)), (int)meta,
                                          (int)nlo, (int)nhi));
    _mm_sfence();
    // (re)launch when no instance runs: never launched, or the last one left
    // on its idle timer (it clears the alive word on its way out, after its
    // last poll -- a request rung after that poll is this one's to serve)
    if (!c.launched || *c.alive() == 0u) rc = c.launch_resident(s - 1u);
  } else {
    const hipError_t e = noise_amd::launch_aead_one(dec, k, nonce, c.d, len, ad_len, s, c.stream);
    if (e != hipSuccess) rc = hip_fail(e, "launch_aead_one");
  }
  std::memset(k, 0, sizeof k);
  if (rc == NOISE_GPU_OK) rc = c.wait(s, res);
  if (rc == NOISE_GPU_OK) {
    std::atomic_thread_fence(std::memory_order_acquire);
    const uint32_t status = dec ? reinterpret_cast<volatile uint32_t *>(c.h)[1] : 0u;
    if (st) *st = status;
    if (!dec) {
      std::memcpy(out, c.h + lay.out, len);
      std::memcpy(out + len, c.h + lay.out + ((len + 15ull) & ~15ull), 16);
    } else if (status == NOISE_GPU_REC_OK) {
      std::memcpy(out, c.h + lay.out, len);
    }
  }
  // hygiene: status, AD, record, output (the resident kernel zeroes its
  // request image itself before the done word; an error path does it here)
  std::memset(c.h + 4, 0, 4);
  if (res) {
    std::memset(c.h + lay.out, 0, lay.total - lay.out);
    if (rc != NOISE_GPU_OK && c.hreq && c.stop_resident() == NOISE_GPU_OK) {
      if (c.req_kind == kReqHost) std::memset(c.hreq, 0, noise_amd::kOneReqBytes);
      else (void)hipMemset(c.dreq, 0, noise_amd::kOneReqBytes);
    }
  } else {
    std::memset(c.h + 128, 0, lay.total - 128);
  }
  return rc;
}

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

namespace noise_amd {
int api_hip_fail(hipError_t e, const char *what) { return hip_fail(e, what); }
int api_arg_fail(const char *msg) { return arg_fail(msg); }
int api_check_device() { return check_device(); }
}  // namespace noise_amd

extern "C" {

const char *noise_gpu_version(void) { return "noise-mi355x 0.1.0 gfx950"; }

const char *noise_gpu_strerror(int status) {
  switch (status) {
    case NOISE_GPU_OK: return "ok";
    case NOISE_GPU_E_NONCE: return "Nonce limit has been exceeded!";
    case NOISE_GPU_E_MAC: return "Invalid MAC";
    case NOISE_GPU_E_ARG: return "invalid argument";
    case NOISE_GPU_E_HIP: return "HIP runtime error";
    case NOISE_GPU_E_NODEV: return "no gfx950 device";
    default: return "unknown status";
  }
}

const char *noise_gpu_last_error(void) { return g_last_error.c_str(); }

int noise_gpu_device_count(int *count) {
  if (!count) return arg_fail("null count");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return NOISE_GPU_OK;
}

int noise_gpu_encrypt_uniform(const uint8_t h_key[32], uint64_t nonce0,
                              const uint8_t *d_in, uint64_t in_stride,
                              uint8_t *d_out, uint64_t out_stride,
                              uint32_t len, const uint8_t *d_ad,
                              uint64_t ad_stride, uint32_t ad_len,
                              uint64_t nrec, void *stream) {
  if (!h_key) return arg_fail("null key");
  int rc = check_uniform(false, d_in, in_stride, d_out, out_stride, len, d_ad,
                         ad_len, nullptr, nrec);
  if (rc || nrec == 0) return rc;
  if (key_absent(h_key)) return arg_fail("all-zero key (no key)");
  if ((rc = check_device())) return rc;
  uint32_t k[8];
  key_words(h_key, k);
  HIP_TRY(noise_amd::launch_aead_uniform(false, k, nonce0, d_in, in_stride,
                                         d_out, out_stride, len, d_ad,
                                         ad_stride, ad_len, nullptr, nrec,
                                         (hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_decrypt_uniform(const uint8_t h_key[32], uint64_t nonce0,
                              const uint8_t *d_in, uint64_t in_stride,
                              uint8_t *d_out, uint64_t out_stride,
                              uint32_t len, const uint8_t *d_ad,
                              uint64_t ad_stride, uint32_t ad_len,
                              uint8_t *d_status, uint64_t nrec, void *stream) {
  if (!h_key) return arg_fail("null key");
  int rc = check_uniform(true, d_in, in_stride, d_out, out_stride, len, d_ad,
                         ad_len, d_status, nrec);
  if (rc || nrec == 0) return rc;
  if (key_absent(h_key)) return arg_fail("all-zero key (no key)");
  if ((rc = check_device())) return rc;
  uint32_t k[8];
  key_words(h_key, k);
  HIP_TRY(noise_amd::launch_aead_uniform(true, k, nonce0, d_in, in_stride,
                                         d_out, out_stride, len, d_ad,
                                         ad_stride, ad_len, d_status, nrec,
                                         (hipStream_t)stream));
  return NOISE_GPU_OK;
}

static int records_dev(bool decrypt, const uint8_t *d_keys, uint32_t nkeys,
                       const noise_gpu_record *d_recs, uint64_t nrec, const uint8_t *d_in,
                       uint8_t *d_out, const uint8_t *d_ad, uint8_t *d_status, uint64_t len_sum,
                       void *stream) {
  if (nrec == 0) return NOISE_GPU_OK;
  if (!d_keys || !nkeys || !d_recs || !d_in || !d_out || (decrypt && !d_status))
    return arg_fail(decrypt ? "null key table / descriptors / buffers / status"
                            : "null key table / descriptors / buffers");
  if (reinterpret_cast<uintptr_t>(d_keys) & 15u)
    return arg_fail("key table must be 16-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::launch_aead_records(decrypt, d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad,
                                         decrypt ? d_status : nullptr, (hipStream_t)stream, len_sum));
  return NOISE_GPU_OK;
}

int noise_gpu_encrypt_records(const uint8_t *d_keys, uint32_t nkeys,
                              const noise_gpu_record *d_recs, uint64_t nrec,
                              const uint8_t *d_in, uint8_t *d_out,
                              const uint8_t *d_ad, void *stream) {
  return records_dev(false, d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad, nullptr, 0, stream);
}

int noise_gpu_decrypt_records(const uint8_t *d_keys, uint32_t nkeys,
                              const noise_gpu_record *d_recs, uint64_t nrec,
                              const uint8_t *d_in, uint8_t *d_out,
                              const uint8_t *d_ad, uint8_t *d_status,
                              void *stream) {
  return records_dev(true, d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad, d_status, 0, stream);
}

int noise_gpu_encrypt_records_sized(const uint8_t *d_keys, uint32_t nkeys,
                                    const noise_gpu_record *d_recs, uint64_t nrec,
                                    const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_ad,
                                    uint64_t len_sum, void *stream) {
  return records_dev(false, d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad, nullptr, len_sum, stream);
}

int noise_gpu_decrypt_records_sized(const uint8_t *d_keys, uint32_t nkeys,
                                    const noise_gpu_record *d_recs, uint64_t nrec,
                                    const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_ad,
                                    uint8_t *d_status, uint64_t len_sum, void *stream) {
  return records_dev(true, d_keys, nkeys, d_recs, nrec, d_in, d_out, d_ad, d_status, len_sum, stream);
}

static int sessions(bool decrypt, const uint8_t *d_keys, uint32_t nkeys,
                    const uint32_t *d_key_idx, const uint64_t *d_nonces,
                    const uint8_t *d_in, uint64_t in_stride, uint8_t *d_out,
                    uint64_t out_stride, uint32_t len, uint8_t *d_status,
                    uint64_t nrec, void *stream) {
  if (nrec == 0) return NOISE_GPU_OK;
  if (!d_keys || !nkeys || !d_key_idx || !d_nonces)
    return arg_fail("null key table / key index / nonce array");
  if (reinterpret_cast<uintptr_t>(d_keys) & 15u)
    return arg_fail("key table must be 16-byte aligned");
  int rc = check_uniform(decrypt, d_in, in_stride, d_out, out_stride, len,
                         nullptr, 0, d_status, nrec);
  if (rc) return rc;
  if (!noise_amd::sessions_supported(len, d_in, in_stride, d_out, out_stride))
    return arg_fail("sessions batches need len in {64,128,192,256,512,1024,2048,4096,8192,16384} "
                    "and 16-byte aligned buffers/strides");
  if ((rc = check_device())) return rc;
  HIP_TRY(noise_amd::launch_aead_sessions(decrypt, d_keys, nkeys, d_key_idx,
                                          d_nonces, d_in, in_stride, d_out,
                                          out_stride, len, d_status, nrec,
                                          (hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_encrypt_sessions(const uint8_t *d_keys, uint32_t nkeys,
                               const uint32_t *d_key_idx,
                               const uint64_t *d_nonces, const uint8_t *d_in,
                               uint64_t in_stride, uint8_t *d_out,
                               uint64_t out_stride, uint32_t len, uint64_t nrec,
                               void *stream) {
  return sessions(false, d_keys, nkeys, d_key_idx, d_nonces, d_in, in_stride,
                  d_out, out_stride, len, nullptr, nrec, stream);
}

int noise_gpu_decrypt_sessions(const uint8_t *d_keys, uint32_t nkeys,
                               const uint32_t *d_key_idx,
                               const uint64_t *d_nonces, const uint8_t *d_in,
                               uint64_t in_stride, uint8_t *d_out,
                               uint64_t out_stride, uint32_t len,
                               uint8_t *d_status, uint64_t nrec, void *stream) {
  return sessions(true, d_keys, nkeys, d_key_idx, d_nonces, d_in, in_stride,
                  d_out, out_stride, len, d_status, nrec, stream);
}

int noise_gpu_rekey_keys(uint8_t *d_keys, uint64_t nkeys, void *stream) {
  if (nkeys == 0) return NOISE_GPU_OK;
  if (!d_keys) return arg_fail("null key table");
  if (reinterpret_cast<uintptr_t>(d_keys) & 15u)
    return arg_fail("key table must be 16-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::launch_rekey(d_keys, nkeys, (hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_x25519(const uint8_t *d_scalars, const uint8_t *d_points,
                     uint8_t *d_out, uint64_t n, void *stream) {
  if (n == 0) return NOISE_GPU_OK;
  if (!d_scalars || !d_out) return arg_fail("null scalars / output");
  if (((reinterpret_cast<uintptr_t>(d_scalars) | reinterpret_cast<uintptr_t>(d_points) |
        reinterpret_cast<uintptr_t>(d_out)) & 15u) != 0)
    return arg_fail("X25519 arrays must be 16-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::launch_x25519(d_scalars, d_points, d_out, n, (hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_scratch_wipe(void *stream) {
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::records_scratch_wipe((hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_scratch_release(void *stream) {
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::records_scratch_release((hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_fill_synthetic(uint8_t *d_dst, uint64_t offset, uint64_t nbytes,
                             uint64_t seed, void *stream) {
  if (nbytes == 0) return NOISE_GPU_OK;
  if (!d_dst) return arg_fail("null destination");
  int rc = check_device();
  if (rc) return rc;
  HIP_TRY(noise_amd::launch_fill_synthetic(d_dst, offset, nbytes, seed,
                                           (hipStream_t)stream));
  return NOISE_GPU_OK;
}

// ---- synchronous host-buffer entry points (CipherState single records)
// Device scratch layout: [ad | pad][record in | pad][record out][status]

int noise_gpu_encrypt_host(const uint8_t h_key[32], uint64_t nonce,
                           const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                           size_t len) {
  if (!h_key || !h_buf || (ad_len && !h_ad))
    return arg_fail("null key / buffer / ad");
  if (key_absent(h_key)) return arg_fail("all-zero key (no key)");
  if (len > 0xffffffffull - 16 || ad_len > 0xffffffffull) return arg_fail("record too large");
  int rc = check_device();
  if (rc) return rc;
  if (ad_len <= noise_amd::kOneMaxAd && len <= 65535)  // latency kernel, mapped staging
    return one_record(false, h_key, nonce, h_ad, (uint32_t)ad_len, h_buf, (uint32_t)len, nullptr,
                      h_buf, nullptr);
  // large AD or record: copy-staged through device scratch, the lane walk
  const size_t ad_sz = align16(ad_len), rec_sz = align16(len + 16);
  NOISE_STAGE(s);
  if ((rc = s.reserve(ad_sz + rec_sz))) return rc;
  std::memcpy(s.h, h_ad, ad_len);
  std::memcpy(s.h + ad_sz, h_buf, len);
  uint32_t k[8];
  key_words(h_key, k);
  hipError_t e = hipMemcpyAsync(s.d, s.h, ad_sz + len, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess)
    e = noise_amd::launch_aead_uniform(false, k, nonce, s.d + ad_sz, 0, s.d + ad_sz, 0,
                                       (uint32_t)len, s.d, 0, (uint32_t)ad_len, nullptr, 1,
                                       s.stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(s.h + ad_sz, s.d + ad_sz, len + 16, hipMemcpyDeviceToHost, s.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  if (e == hipSuccess) std::memcpy(h_buf, s.h + ad_sz, len + 16);
  std::memset(k, 0, sizeof k);
  s.wipe(ad_sz + rec_sz);
  return e == hipSuccess ? NOISE_GPU_OK : hip_fail(e, "encrypt_host (staged)");
}

int noise_gpu_decrypt_host(const uint8_t h_key[32], uint64_t nonce,
                           const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                           size_t ct_len) {
  if (!h_key || !h_buf || (ad_len && !h_ad))
    return arg_fail("null key / buffer / ad");
  if (key_absent(h_key)) return arg_fail("all-zero key (no key)");
  if (ct_len < 16) {  // reference UB (noise.cpp:257); defined as bad MAC
    g_last_error = "ciphertext shorter than the tag";
    return NOISE_GPU_E_MAC;
  }
  if (ct_len > 0xffffffffull || ad_len > 0xffffffffull) return arg_fail("record too large");
  int rc = check_device();
  if (rc) return rc;
  const size_t len = ct_len - 16;
  uint32_t st = NOISE_GPU_REC_BAD_MAC;
  if (ad_len <= noise_amd::kOneMaxAd && len <= 65535) {
    rc = one_record(true, h_key, nonce, h_ad, (uint32_t)ad_len, h_buf, (uint32_t)len,
                    h_buf + len, h_buf, &st);
  } else {  // large AD or record: copy-staged through device scratch, the lane walk
    const size_t ad_sz = align16(ad_len), in_sz = align16(ct_len), out_sz = align16(len);
    NOISE_STAGE(s);
    if ((rc = s.reserve(ad_sz + in_sz + out_sz + 16))) return rc;
    uint8_t *d_in = s.d + ad_sz, *d_out = d_in + in_sz, *d_st = d_out + out_sz;
    std::memcpy(s.h, h_ad, ad_len);
    std::memcpy(s.h + ad_sz, h_buf, ct_len);
    uint32_t k[8];
    key_words(h_key, k);
    uint8_t *h_out = s.h + ad_sz + in_sz;
    hipError_t e = hipMemcpyAsync(s.d, s.h, ad_sz + ct_len, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = noise_amd::launch_aead_uniform(true, k, nonce, d_in, 0, d_out, 0, (uint32_t)len, s.d, 0,
                                         (uint32_t)ad_len, d_st, 1, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h_out, d_out, out_sz + 16, hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
    std::memset(k, 0, sizeof k);
    if (e == hipSuccess) {
      st = h_out[out_sz];
      if (st == NOISE_GPU_REC_OK) std::memcpy(h_buf, h_out, len);
    }
    s.wipe(ad_sz + in_sz + out_sz + 16);
    rc = e == hipSuccess ? NOISE_GPU_OK : hip_fail(e, "decrypt_host (staged)");
  }
  if (rc) return rc;
  if (st != NOISE_GPU_REC_OK) {
    g_last_error = "Invalid MAC";
    return NOISE_GPU_E_MAC;
  }
  return NOISE_GPU_OK;
}

int noise_gpu_rekey_host(uint8_t h_key[32]) {
  // k <- ENCRYPT(k, 2^64-2, empty, 0^32)[0..32) (noise.cpp:429-439)
  if (!h_key) return arg_fail("null key");
  int rc = check_device();
  if (rc) return rc;
  uint8_t zero[32] = {0}, out[48];
  rc = one_record(false, h_key, ~0ull - 1ull, nullptr, 0, zero, 32, nullptr, out, nullptr);
  if (rc == NOISE_GPU_OK) std::memcpy(h_key, out, 32);
  std::memset(out, 0, sizeof out);
  return rc;
}

// ---- host descriptor batches (CipherState::encrypt_batch/decrypt_batch)
static int records_host(bool decrypt, const uint8_t *h_keys, uint32_t nkeys,
                        const noise_gpu_record *h_recs, uint64_t nrec,
                        const uint8_t *h_in, uint64_t in_bytes, uint8_t *h_out,
                        uint64_t out_bytes, const uint8_t *h_ad,
                        uint64_t ad_bytes, uint8_t *h_status) {
  if (nrec == 0) return NOISE_GPU_OK;
  if (!h_keys || !nkeys || !h_recs || (in_bytes && !h_in) ||
      (out_bytes && !h_out) || (ad_bytes && !h_ad) || (decrypt && !h_status))
    return arg_fail("null key table / descriptors / buffers");
  for (uint64_t i = 0; i < nrec; ++i) {  // host-side bounds check of every record
    const noise_gpu_record &r = h_recs[i];
    const uint64_t in_len = decrypt ? (uint64_t)r.len + 16 : r.len;
    const uint64_t out_len = decrypt ? r.len : (uint64_t)r.len + 16;
    // overflow-safe: an offset near 2^64 must not wrap past the check
    if (r.key_idx >= nkeys || in_len > in_bytes || r.in_off > in_bytes - in_len ||
        out_len > out_bytes || r.out_off > out_bytes - out_len ||
        (r.ad_len && (r.ad_len > ad_bytes || r.ad_off > ad_bytes - r.ad_len)))
      return arg_fail("record descriptor out of range");
  }
  int rc = check_device();
  if (rc) return rc;
  const size_t o_keys = 0, o_recs = align16(32ull * nkeys),
               o_in = o_recs + align16(sizeof(noise_gpu_record) * nrec),
               o_out = o_in + align16(in_bytes), o_ad = o_out + align16(out_bytes),
               o_st = o_ad + align16(ad_bytes), total = o_st + align16(nrec);
  NOISE_STAGE(s);
  if ((rc = s.reserve(total))) return rc;
  std::memcpy(s.h + o_keys, h_keys, 32ull * nkeys);
  std::memcpy(s.h + o_recs, h_recs, sizeof(noise_gpu_record) * nrec);
  if (in_bytes) std::memcpy(s.h + o_in, h_in, in_bytes);
  if (ad_bytes) std::memcpy(s.h + o_ad, h_ad, ad_bytes);
  hipError_t e = hipMemcpyAsync(s.d, s.h, o_out, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess && ad_bytes)
    e = hipMemcpyAsync(s.d + o_ad, s.h + o_ad, ad_bytes, hipMemcpyHostToDevice, s.stream);
  uint64_t len_sum = 0;  // the descriptors are on the host here: the batch's size
  for (uint64_t i = 0; i < nrec; ++i) len_sum += h_recs[i].len;
  if (e == hipSuccess)
    e = noise_amd::launch_aead_records(
        decrypt, s.d + o_keys, nkeys,
        reinterpret_cast<const noise_gpu_record *>(s.d + o_recs), nrec, s.d + o_in,
        s.d + o_out, s.d + o_ad, decrypt ? s.d + o_st : nullptr, s.stream, len_sum);
  if (e == hipSuccess)
    e = hipMemcpyAsync(s.h + o_out, s.d + o_out, o_st + nrec - o_out, hipMemcpyDeviceToHost,
                       s.stream);
  if (e == hipSuccess) e = noise_amd::records_scratch_wipe(s.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  if (e == hipSuccess) {
    if (out_bytes) std::memcpy(h_out, s.h + o_out, out_bytes);
    if (decrypt) std::memcpy(h_status, s.h + o_st, nrec);
  }
  s.wipe(total);  // keys, plaintext, ciphertext: host image and device scratch
  return e == hipSuccess ? NOISE_GPU_OK : hip_fail(e, "records_host");
}

int noise_gpu_encrypt_records_host(const uint8_t *h_keys, uint32_t nkeys,
                                   const noise_gpu_record *h_recs,
                                   uint64_t nrec, const uint8_t *h_in,
                                   uint64_t in_bytes, uint8_t *h_out,
                                   uint64_t out_bytes, const uint8_t *h_ad,
                                   uint64_t ad_bytes) {
  return records_host(false, h_keys, nkeys, h_recs, nrec, h_in, in_bytes,
                      h_out, out_bytes, h_ad, ad_bytes, nullptr);
}

int noise_gpu_decrypt_records_host(const uint8_t *h_keys, uint32_t nkeys,
                                   const noise_gpu_record *h_recs,
                                   uint64_t nrec, const uint8_t *h_in,
                                   uint64_t in_bytes, uint8_t *h_out,
                                   uint64_t out_bytes, const uint8_t *h_ad,
                                   uint64_t ad_bytes, uint8_t *h_status) {
  return records_host(true, h_keys, nkeys, h_recs, nrec, h_in, in_bytes, h_out,
                      out_bytes, h_ad, ad_bytes, h_status);
}

// ---- host-resident uniform batches: chunked 3-stream pipeline ----------
// Streams and device chunk buffers persist per (thread, device); a call
// pays only its copies and kernels (and the wipe of the chunks it used).
namespace {
struct PipeCtx {
  static constexpr int kDepth = 3;
  static constexpr uint64_t kChunk = 32ull << 20;  // bytes in + out per chunk
  int dev = -1;
  hipStream_t st[kDepth] = {};
  uint8_t *buf[kDepth] = {};  // [in | out | status] of one chunk
  ~PipeCtx() { release(); }
  void release() {
    for (int i = 0; i < kDepth; ++i) {
      if (buf[i]) (void)noise_amd::dev_wipe_free(buf[i], kChunk + (kChunk >> 4), st[i]);
      if (st[i]) (void)hipStreamSynchronize(st[i]);
      if (st[i]) (void)hipStreamDestroy(st[i]);
      buf[i] = nullptr;
      st[i] = nullptr;
    }
    dev = -1;
  }
  int ready() {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    if (cur == dev) return NOISE_GPU_OK;
    release();
    for (int i = 0; i < kDepth; ++i) {
      HIP_TRY(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
      HIP_TRY(noise_amd::dev_alloc(reinterpret_cast<void **>(&buf[i]), kChunk + (kChunk >> 4), st[i]));
    }
    dev = cur;
    return NOISE_GPU_OK;
  }
};
thread_local PipeCtx g_pipe_tab[kMaxCtxDev];
thread_local PipeCtx *tl_pipe = nullptr;
}  // namespace

static int uniform_host(bool decrypt, const uint8_t h_key[32], uint64_t nonce0,
                        const uint8_t *h_in, uint64_t in_stride, uint8_t *h_out,
                        uint64_t out_stride, uint32_t len, uint8_t *h_status,
                        uint64_t nrec, double *seconds) {
  const auto t0 = std::chrono::steady_clock::now();  // the whole call is timed
  if (!h_key) return arg_fail("null key");
  if (key_absent(h_key)) return arg_fail("all-zero key (no key)");
  int rc = check_uniform(decrypt, h_in, in_stride, h_out, out_stride, len,
                         nullptr, 0, decrypt ? (const void *)h_status : h_in,
                         nrec);
  if (rc) return rc;
  if (h_in == h_out) return arg_fail("host batches must be out-of-place");
  if (len > NOISE_GPU_UNIFORM_HOST_MAX_LEN)
    return arg_fail("record longer than NOISE_GPU_UNIFORM_HOST_MAX_LEN for the host pipeline");
  if (nrec == 0) {
    if (seconds) *seconds = 0;
    return NOISE_GPU_OK;
  }
  if ((rc = check_device())) return rc;
  PipeCtx *pp = tl_pipe ? tl_pipe : ctx_of(g_pipe_tab);
  if (!pp) return hip_fail(hipErrorInvalidDevice, "hipGetDevice");
  if ((rc = pp->ready())) return rc;
  PipeCtx &P = *pp;
  const uint64_t in_rec = decrypt ? (uint64_t)len + 16 : len;
  const uint64_t out_rec = decrypt ? len : (uint64_t)len + 16;
  // device chunks are packed (stride = record size), ~32 MiB of in + out
  static_assert(2ull * NOISE_GPU_UNIFORM_HOST_MAX_LEN + 17 <= PipeCtx::kChunk,
                "a chunk holds at least one record of the documented maximum");
  const uint64_t per = std::max<uint64_t>(1, PipeCtx::kChunk / (in_rec + out_rec + 1));
  if (per * (in_rec + out_rec) + per > PipeCtx::kChunk + (PipeCtx::kChunk >> 4))
    return arg_fail("record too large for the host pipeline");
  uint32_t k[8];
  key_words(h_key, k);
  hipError_t e = hipSuccess;
  uint64_t used[PipeCtx::kDepth] = {0, 0, 0};
  for (uint64_t first = 0, c = 0; first < nrec && e == hipSuccess; first += per, ++c) {
    const uint64_t n = std::min(per, nrec - first);
    const int b = (int)(c % PipeCtx::kDepth);
    uint8_t *d_in = P.buf[b], *d_out = d_in + per * in_rec, *d_stat = d_out + per * out_rec;
    used[b] = std::max(used[b], per * (in_rec + out_rec) + per);
    e = hipMemcpy2DAsync(d_in, in_rec, h_in + first * in_stride, in_stride,
                         in_rec, n, hipMemcpyHostToDevice, P.st[b]);
    if (e == hipSuccess)
      e = noise_amd::launch_aead_uniform(decrypt, k, nonce0 + first, d_in,
                                         in_rec, d_out, out_rec, len,
                                         nullptr, 0, 0, decrypt ? d_stat : nullptr, n, P.st[b]);
    if (e == hipSuccess)
      e = hipMemcpy2DAsync(h_out + first * out_stride, out_stride, d_out,
                           out_rec, out_rec, n, hipMemcpyDeviceToHost, P.st[b]);
    if (e == hipSuccess && decrypt)
      e = hipMemcpyAsync(h_status + first, d_stat, n, hipMemcpyDeviceToHost, P.st[b]);
  }
  std::memset(k, 0, sizeof k);
  for (int i = 0; i < PipeCtx::kDepth && e == hipSuccess; ++i) e = hipStreamSynchronize(P.st[i]);
  const auto t1 = std::chrono::steady_clock::now();
  // hygiene: the chunks held plaintext and ciphertext
  for (int i = 0; i < PipeCtx::kDepth; ++i)
    if (used[i]) (void)hipMemsetAsync(P.buf[i], 0, used[i], P.st[i]);
  if (e != hipSuccess) {
    P.release();
    return hip_fail(e, "host pipeline");
  }
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  return NOISE_GPU_OK;
}

int noise_gpu_encrypt_uniform_host(const uint8_t h_key[32], uint64_t nonce0,
                                   const uint8_t *h_in, uint64_t in_stride,
                                   uint8_t *h_out, uint64_t out_stride,
                                   uint32_t len, uint64_t nrec,
                                   double *seconds) {
  return uniform_host(false, h_key, nonce0, h_in, in_stride, h_out, out_stride,
                      len, nullptr, nrec, seconds);
}

int noise_gpu_decrypt_uniform_host(const uint8_t h_key[32], uint64_t nonce0,
                                   const uint8_t *h_in, uint64_t in_stride,
                                   uint8_t *h_out, uint64_t out_stride,
                                   uint32_t len, uint8_t *h_status,
                                   uint64_t nrec, double *seconds) {
  return uniform_host(true, h_key, nonce0, h_in, in_stride, h_out, out_stride,
                      len, h_status, nrec, seconds);
}


// ---- explicit device contexts -------------------------------------------
// A noise_gpu_ctx owns the host-entry-point contexts (staging, latency
// path, pipeline) of one device.  Its entry points make that device current
// and the ctx's contexts the thread's for the duration of the call, then
// restore both.
}  // extern "C"

struct noise_gpu_ctx {
  int device = -1;
  Staging stage;
  OneCtx one;
  PipeCtx pipe;
};

namespace {
struct CtxScope {
  int prev = -1;
  Staging *s0;
  OneCtx *o0;
  PipeCtx *p0;
  int rc = NOISE_GPU_OK;
  explicit CtxScope(noise_gpu_ctx *c) : s0(tl_stage), o0(tl_one), p0(tl_pipe) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    const hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) {
      rc = hip_fail(e, "hipSetDevice(ctx device)");
      return;
    }
    tl_stage = &c->stage;
    tl_one = &c->one;
    tl_pipe = &c->pipe;
  }
  ~CtxScope() {
    tl_stage = s0;
    tl_one = o0;
    tl_pipe = p0;
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace

#define NOISE_CTX_CALL(ctx, call)                                              \
  do {                                                                         \
    if (!(ctx)) return arg_fail("null context");                               \
    CtxScope scope_(ctx);                                                      \
    if (scope_.rc) return scope_.rc;                                           \
    return call;                                                               \
  } while (0)

extern "C" {

static int set_resident(OneCtx &c, int on, uint32_t idle_us) {
  if (idle_us > kResidentIdleMaxUs) return arg_fail("idle_us above 10 s");
  if (on) {
    int rc = check_device();
    if (rc) return rc;
    c.idle_us = idle_us ? idle_us : kResidentIdleDefaultUs;
    if (c.resident)  // new idle time: the next instance takes it
      return c.stop_resident();
    c.resident = true;
    return NOISE_GPU_OK;
  }
  if (int rc = c.stop_resident()) return rc;  // wedged: the image stays (the kernel reads it)
  c.release_req();  // zeroed and freed: nothing of the mode stays behind
  c.resident = false;
  return NOISE_GPU_OK;
}

int noise_gpu_set_resident(int on, uint32_t idle_us) {
  OneCtx *cp = tl_one ? tl_one : ctx_of(g_one_tab);
  if (!cp) return hip_fail(hipErrorInvalidDevice, "hipGetDevice");
  return set_resident(*cp, on, idle_us);
}

int noise_gpu_thread_release(void) {
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  for (int i = 0; i < kMaxCtxDev; ++i) {
    g_stage_tab[i].release();
    g_one_tab[i].release();
    g_pipe_tab[i].release();
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return NOISE_GPU_OK;
}

int noise_gpu_ctx_create(int device, noise_gpu_ctx **out) {
  if (!out) return arg_fail("null output pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    g_last_error = "no HIP device visible";
    return NOISE_GPU_E_NODEV;
  }
  if (device < 0 || device >= n) return arg_fail("device index out of range");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  HIP_TRY(hipSetDevice(device));
  const int rc = check_device();  // gfx950 only
  if (prev >= 0) (void)hipSetDevice(prev);
  if (rc) return rc;
  noise_gpu_ctx *c = new (std::nothrow) noise_gpu_ctx;
  if (!c) return arg_fail("out of host memory");
  c->device = device;
  *out = c;
  return NOISE_GPU_OK;
}

int noise_gpu_ctx_destroy(noise_gpu_ctx *ctx) {
  if (!ctx) return NOISE_GPU_OK;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  (void)hipSetDevice(ctx->device);
  delete ctx;  // the contexts wipe what they staged, then free it
  if (prev >= 0) (void)hipSetDevice(prev);
  return NOISE_GPU_OK;
}

int noise_gpu_ctx_set_resident(noise_gpu_ctx *ctx, int on, uint32_t idle_us) {
  NOISE_CTX_CALL(ctx, set_resident(ctx->one, on, idle_us));
}

int noise_gpu_ctx_device(const noise_gpu_ctx *ctx, int *device) {
  if (!ctx || !device) return arg_fail("null argument");
  *device = ctx->device;
  return NOISE_GPU_OK;
}

int noise_gpu_ctx_encrypt_host(noise_gpu_ctx *ctx, const uint8_t h_key[32], uint64_t nonce,
                               const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf, size_t len) {
  NOISE_CTX_CALL(ctx, noise_gpu_encrypt_host(h_key, nonce, h_ad, ad_len, h_buf, len));
}

int noise_gpu_ctx_decrypt_host(noise_gpu_ctx *ctx, const uint8_t h_key[32], uint64_t nonce,
                               const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                               size_t ct_len) {
  NOISE_CTX_CALL(ctx, noise_gpu_decrypt_host(h_key, nonce, h_ad, ad_len, h_buf, ct_len));
}

int noise_gpu_ctx_rekey_host(noise_gpu_ctx *ctx, uint8_t h_key[32]) {
  NOISE_CTX_CALL(ctx, noise_gpu_rekey_host(h_key));
}

int noise_gpu_ctx_encrypt_records_host(noise_gpu_ctx *ctx, const uint8_t *h_keys, uint32_t nkeys,
                                       const noise_gpu_record *h_recs, uint64_t nrec,
                                       const uint8_t *h_in, uint64_t in_bytes, uint8_t *h_out,
                                       uint64_t out_bytes, const uint8_t *h_ad,
                                       uint64_t ad_bytes) {
  NOISE_CTX_CALL(ctx, noise_gpu_encrypt_records_host(h_keys, nkeys, h_recs, nrec, h_in, in_bytes,
                                                     h_out, out_bytes, h_ad, ad_bytes));
}

int noise_gpu_ctx_decrypt_records_host(noise_gpu_ctx *ctx, const uint8_t *h_keys, uint32_t nkeys,
                                       const noise_gpu_record *h_recs, uint64_t nrec,
                                       const uint8_t *h_in, uint64_t in_bytes, uint8_t *h_out,
                                       uint64_t out_bytes, const uint8_t *h_ad,
                                       uint64_t ad_bytes, uint8_t *h_status) {
  NOISE_CTX_CALL(ctx, noise_gpu_decrypt_records_host(h_keys, nkeys, h_recs, nrec, h_in, in_bytes,
                                                     h_out, out_bytes, h_ad, ad_bytes, h_status));
}

int noise_gpu_ctx_encrypt_uniform_host(noise_gpu_ctx *ctx, const uint8_t h_key[32],
                                       uint64_t nonce0, const uint8_t *h_in, uint64_t in_stride,
                                       uint8_t *h_out, uint64_t out_stride, uint32_t len,
                                       uint64_t nrec, double *seconds) {
  NOISE_CTX_CALL(ctx, uniform_host(false, h_key, nonce0, h_in, in_stride, h_out, out_stride, len,
                                   nullptr, nrec, seconds));
}

int noise_gpu_ctx_decrypt_uniform_host(noise_gpu_ctx *ctx, const uint8_t h_key[32],
                                       uint64_t nonce0, const uint8_t *h_in, uint64_t in_stride,
                                       uint8_t *h_out, uint64_t out_stride, uint32_t len,
                                       uint8_t *h_status, uint64_t nrec, double *seconds) {
  NOISE_CTX_CALL(ctx, uniform_host(true, h_key, nonce0, h_in, in_stride, h_out, out_stride, len,
                                   h_status, nrec, seconds));
}
}  // extern "C"
