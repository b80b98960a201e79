// emu_records.cpp -- run the engine's descriptor-batch path
// (noise_amd::launch_aead_records: classification, tile / wave / generic
// kernels) on the CPU through the HIP stand-in (include/hip/hip_runtime.h),
// under AddressSanitizer, against the C oracle.  Buffers are malloc'd at
// their exact sizes, so any access outside a record's extent is reported.
//
//   emu_records <mode> <nrec> <seed>
//     mode cfg4   : BASELINE config-4 lengths (64 * 2^k, P(k) ~ 1/(k+1),
//                   top bucket 65519), packed 16-byte aligned, one key,
//                   out-of-place encrypt + decrypt + tamper
//     mode inplace: same lengths, encrypt and decrypt in place
//     mode ragged : lengths uniform in 1..70000 (odd tails, > 65535 generic)
//     mode jitter : config-4 buckets minus U(0..63) bytes (the masked tile
//                   classes and masked tail units); jitterinplace: in place
//   emu_records <mode> <nrec> <seed> <gap>: records start <gap> bytes into
//     each buffer (e.g. 4 GiB, to exercise 64-bit offsets)
// Test infrastructure only (links oracle/chachapoly_oracle.c).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "launchers.hpp"

extern "C" {
void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                          size_t ad_len, const uint8_t *pt, size_t len, uint8_t *out);
int oracle_noise_decrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                         size_t ad_len, const uint8_t *ct, size_t ct_len, uint8_t *out);
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Decrypt with the store hook on: no store may put a non-zero byte into the
// output range of a record whose tag fails, nor any store at all into one
// decrypted in place (crypto_aead_read, monocypher.c:2912-2929: plaintext is
// written only after the tag has verified).  Ranges sorted by start.
struct Range {
  uintptr_t lo, hi;
};
static std::vector<Range> g_bad_ranges;
static bool g_bad_in_place = false;
static std::atomic<long> g_bad_stores{0}, g_bad_first{-1};
static uintptr_t g_out_lo = 0, g_out_hi = 0;  // the decrypt's output buffer
static std::atomic<long> g_out_of_range{0};
static void watch_store(const void *dst, const void *data, int n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst), b = a + (uintptr_t)n;
  if (a < g_out_lo || b > g_out_hi) {  // reported, and not performed by ASan either
    if (g_out_of_range.fetch_add(1) < 5)
      std::printf("store outside the output buffer: offset %lld, %d bytes\n",
                  (long long)(a - g_out_lo), n);
    std::fflush(stdout);
    std::abort();
  }
  auto it = std::upper_bound(g_bad_ranges.begin(), g_bad_ranges.end(), a,
                             [](uintptr_t x, const Range &r) { return x < r.lo; });
  // the range starting at or before a, and the next one (a store may straddle)
  for (int k = 0; k < 2; ++k) {
    const Range *r = nullptr;
    if (k == 0 && it != g_bad_ranges.begin()) r = &*(it - 1);
    if (k == 1 && it != g_bad_ranges.end()) r = &*it;
    if (!r || b <= r->lo || a >= r->hi) continue;
    bool bad = g_bad_in_place;
    const uint8_t *p = static_cast<const uint8_t *>(data);
    for (int i = 0; i < n && !bad; ++i)
      if (a + (uintptr_t)i >= r->lo && a + (uintptr_t)i < r->hi && p[i] != 0) bad = true;
    if (bad && g_bad_stores.fetch_add(1) == 0) g_bad_first = (long)(a - r->lo);
  }
}

static int fails = 0;
#define CHECK(c, ...)                        \
  do {                                       \
    if (!(c)) {                              \
      if (fails < 20) {                      \
        std::printf("FAIL: " __VA_ARGS__);   \
        std::printf("\n");                   \
      }                                      \
      ++fails;                               \
    }                                        \
  } while (0)

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "cfg4";
  const uint64_t R = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 3000;
  const uint64_t seed = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 4;
  const bool in_place = std::strcmp(mode, "inplace") == 0 || std::strcmp(mode, "jitterinplace") == 0;
  const bool ragged = std::strcmp(mode, "ragged") == 0;
  // jitter: config-4 buckets, each length lowered by U(0..63) (bench.py --jitter)
  const bool jitter = std::strcmp(mode, "jitter") == 0 || std::strcmp(mode, "jitterinplace") == 0;
  const uint64_t gap = argc > 4 ? std::strtoull(argv[4], nullptr, 0) : 0;

  double w[11], tot = 0;
  for (int k = 0; k < 11; ++k) tot += (w[k] = 1.0 / (k + 1));
  std::vector<uint32_t> lens(R);
  for (uint64_t i = 0; i < R; ++i) {
    const double u = (double)mix64(seed + (i + 1) * 0x9e3779b97f4a7c15ull) / 18446744073709551616.0;
    double c = 0;
    int k = 0;
    for (; k < 10; ++k) {
      c += w[k] / tot;
      if (u < c) break;
    }
    lens[i] = k == 10 ? 65519u : (64u << k);
    if (jitter) lens[i] = std::min(65519u, (64u << k) - (uint32_t)(mix64(seed * 3 + i) % 64u));
    if (ragged) lens[i] = 1u + (uint32_t)(mix64(seed * 7 + i) % 70000u);  // long tails, > 65535
  }
  std::vector<noise_gpu_record> enc(R), dec(R);
  uint64_t in_off = gap, ct_off = gap;
  for (uint64_t i = 0; i < R; ++i) {
    const uint64_t L = lens[i];
    const uint64_t in_sz = (L + 15) / 16 * 16, ct_sz = (L + 31) / 16 * 16;
    enc[i] = noise_gpu_record{in_off, ct_off, 1000 + i, 0, (uint32_t)L, 0, 0, 0};
    if (in_place) enc[i].out_off = enc[i].in_off = ct_off;
    dec[i] = enc[i];
    dec[i].in_off = enc[i].out_off;
    dec[i].out_off = enc[i].in_off;
    in_off += in_sz;
    ct_off += ct_sz;
  }
  const uint64_t tot_in = in_place ? ct_off : in_off, tot_ct = ct_off;
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
  uint8_t *pt = (uint8_t *)std::malloc(tot_in);
  for (uint64_t j = gap; j < tot_in; ++j) pt[j] = (uint8_t)mix64(j * 31 + seed);
  uint8_t *ct = in_place ? pt : (uint8_t *)std::malloc(tot_ct);
  std::vector<uint8_t> pt_copy(tot_in - gap);
  std::memcpy(pt_copy.data(), pt + gap, tot_in - gap);

  // descriptors / keys in "device" memory of exact size
  noise_gpu_record *d_enc = (noise_gpu_record *)std::malloc(R * sizeof(noise_gpu_record));
  noise_gpu_record *d_dec = (noise_gpu_record *)std::malloc(R * sizeof(noise_gpu_record));
  std::memcpy(d_enc, enc.data(), R * sizeof(noise_gpu_record));
  std::memcpy(d_dec, dec.data(), R * sizeof(noise_gpu_record));
  uint8_t *d_key = (uint8_t *)std::malloc(32);
  std::memcpy(d_key, key, 32);

  hipError_t e = noise_amd::launch_aead_records(false, d_key, 1, d_enc, R, pt, ct, nullptr, nullptr, nullptr);
  CHECK(e == hipSuccess, "encrypt launch %d", e);
  std::vector<uint8_t> want(70000 + 16);
  for (uint64_t i = 0; i < R; ++i) {
    const uint32_t L = lens[i];
    oracle_noise_encrypt(key, enc[i].nonce, nullptr, 0, pt_copy.data() + (enc[i].in_off - gap), L, want.data());
    CHECK(std::memcmp(ct + enc[i].out_off, want.data(), L + 16) == 0, "encrypt record %llu len %u",
          (unsigned long long)i, L);
  }
  // tamper a few records of each kind
  std::vector<uint8_t> bad(R, 0);
  for (uint64_t i = 0; i < R; i += 97) {
    ct[enc[i].out_off + (i * 13) % (lens[i] + 16)] ^= 0x10;
    bad[i] = 1;
  }
  std::vector<uint8_t> ct_copy(tot_ct - gap);
  std::memcpy(ct_copy.data(), ct + gap, tot_ct - gap);
  uint8_t *back = in_place ? ct : (uint8_t *)std::malloc(tot_in);
  if (!in_place) std::memset(back + gap, 0xC3, tot_in - gap);
  uint8_t *st = (uint8_t *)std::malloc(R);
  std::memset(st, 9, R);
  for (uint64_t i = 0; i < R; ++i)
    if (bad[i])
      g_bad_ranges.push_back(Range{reinterpret_cast<uintptr_t>(back + dec[i].out_off),
                                   reinterpret_cast<uintptr_t>(back + dec[i].out_off) + lens[i]});
  std::sort(g_bad_ranges.begin(), g_bad_ranges.end(), [](const Range &x, const Range &y) { return x.lo < y.lo; });
  g_bad_in_place = in_place;
  g_out_lo = reinterpret_cast<uintptr_t>(back);
  g_out_hi = g_out_lo + tot_in;
  emu::store_hook = watch_store;
  e = noise_amd::launch_aead_records(true, d_key, 1, d_dec, R, ct, back, nullptr, st, nullptr);
  emu::store_hook = nullptr;
  CHECK(e == hipSuccess, "decrypt launch %d", e);
  CHECK(g_bad_stores.load() == 0, "%ld stores of unverified plaintext into failed records (first at byte %ld)",
        g_bad_stores.load(), g_bad_first.load());
  std::printf("watched %zu failed records: %ld stores of unverified plaintext\n", g_bad_ranges.size(),
              g_bad_stores.load());
  for (uint64_t i = 0; i < R; ++i) {
    const uint32_t L = lens[i];
    if (bad[i]) {
      CHECK(st[i] == 1, "status of tampered record %llu len %u = %u", (unsigned long long)i, L, st[i]);
      if (in_place)
        CHECK(std::memcmp(back + dec[i].out_off, ct_copy.data() + (dec[i].in_off - gap), L + 16) == 0,
              "in-place failure modified record %llu", (unsigned long long)i);
      else
        for (uint32_t b = 0; b < L; ++b)
          if (back[dec[i].out_off + b] != 0) {
            CHECK(false, "failed copy not zeroed %llu", (unsigned long long)i);
            break;
          }
    } else {
      CHECK(st[i] == 0, "status of record %llu len %u = %u", (unsigned long long)i, L, st[i]);
      {
        uint32_t bad = 0, first = L, nbad = 0;
        for (uint32_t b = 0; b < L; ++b)
          if (back[dec[i].out_off + b] != pt_copy[enc[i].in_off - gap + b]) {
            if (first == L) first = b;
            ++nbad;
          }
        bad = nbad;
        CHECK(bad == 0, "decrypt record %llu len %u (%u bytes differ, first at %u)", (unsigned long long)i, L,
              nbad, first);
      }
    }
  }
  std::printf("%s R=%llu bytes=%llu: %s (%d failures)\n", mode, (unsigned long long)R,
              (unsigned long long)tot_in, fails ? "FAIL" : "ok", fails);
  std::free(pt);
  if (!in_place) {
    std::free(ct);
    std::free(back);
  }
  std::free(st);
  std::free(d_enc);
  std::free(d_dec);
  std::free(d_key);
  return fails ? 1 : 0;
}
