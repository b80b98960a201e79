// emu_uniform.cpp -- the uniform-batch entry (noise_amd::launch_aead_uniform)
// for record lengths off the exact tile table: 16-byte aligned strides and
// any length 1..16384 take the masked tile kernel (csrc/mtile_kernel.hpp).
// Run on the CPU through the HIP stand-in under AddressSanitizer, against
// the C oracle, with every store watched:
//   * encrypt: every record's ct || tag equals the oracle's; nothing outside
//     [out + i*stride, + len + 16) is written (canary bytes in the gaps);
//   * decrypt of a batch with tampered records (tag, first, last ciphertext
//     byte): status per record; verified records' plaintext exact; a failed
//     record gets no store at all in place, zeros as a copy; no store past
//     [out + i*stride, + len) -- no byte of unverified plaintext is stored.
//   emu_uniform <seed> <len>...      (default: the length list below)
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
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static int fails = 0;
#define CHECK(c, ...)                        \
  do {                                       \
    if (!(c)) {                              \
      if (fails < 30) {                      \
        std::printf("FAIL: " __VA_ARGS__);   \
        std::printf("\n");                   \
      }                                      \
      ++fails;                               \
    }                                        \
  } while (0)

// store watch: [lo, hi) is the output extent of record i; `bad` records must
// get no store (in place) or only zero bytes (copy)
struct Ext {
  uintptr_t lo, hi;
  bool bad;
};
static std::vector<Ext> g_ext;
static bool g_inplace = false;
static std::atomic<long> g_outside{0}, g_unverified{0};
static void watch(const void *dst, const void *data, int n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst), b = a + (uintptr_t)n;
  auto it = std::upper_bound(g_ext.begin(), g_ext.end(), a, [](uintptr_t x, const Ext &e) { return x < e.lo; });
  if (it == g_ext.begin() || b > (it - 1)->hi) {
    if (g_outside.fetch_add(1) < 5) std::printf("store outside every record's output: %d bytes\n", n);
    return;
  }
  const Ext &e = *(it - 1);
  if (!e.bad) return;
  bool nz = g_inplace;
  for (int i = 0; i < n && !nz; ++i) nz = static_cast<const uint8_t *>(data)[i] != 0;
  if (nz) g_unverified.fetch_add(1);
}

static void run(uint32_t L, uint64_t seed, bool inplace, uint64_t R) {
  const uint64_t c16 = (L + 15) / 16 * 16, ct16 = (L + 31) / 16 * 16;
  // padded strides: records start 16-byte aligned, with gaps after them
  const uint64_t sin = inplace ? ct16 + 32 : c16 + 16 * (seed % 3), sct = inplace ? sin : ct16 + 32;
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(mix64(seed + i) | 1);
  uint32_t k[8];
  std::memcpy(k, key, 32);
  const uint64_t nonce0 = mix64(seed * 5 + L) & 0xffffffffull;
  // exact-size buffers (ASan): the masked kernel reads whole 16-byte pieces,
  // so the buffers end on a 16-byte boundary, as any allocation does on the GPU
  std::vector<uint8_t> pt_ref(R * L);
  for (uint64_t j = 0; j < R * L; ++j) pt_ref[j] = (uint8_t)mix64(seed * 131 + j);
  uint8_t *pt = (uint8_t *)std::aligned_alloc(16, R * sin);
  uint8_t *ct = inplace ? pt : (uint8_t *)std::aligned_alloc(16, R * sct);
  std::memset(pt, 0xA5, R * sin);
  if (!inplace) std::memset(ct, 0x5A, R * sct);
  for (uint64_t i = 0; i < R; ++i) std::memcpy(pt + i * sin, pt_ref.data() + i * L, L);

  g_ext.clear();
  for (uint64_t i = 0; i < R; ++i)
    g_ext.push_back(Ext{reinterpret_cast<uintptr_t>(ct + i * sct), reinterpret_cast<uintptr_t>(ct + i * sct) + L + 16, false});
  g_inplace = false;
  emu::store_hook = watch;
  hipError_t e = noise_amd::launch_aead_uniform(false, k, nonce0, pt, sin, ct, sct, L, nullptr, 0, 0, nullptr, R, nullptr);
  emu::store_hook = nullptr;
  CHECK(e == hipSuccess, "encrypt launch L=%u", L);
  std::vector<uint8_t> want(L + 16);
  for (uint64_t i = 0; i < R; ++i) {
    oracle_noise_encrypt(key, nonce0 + i, nullptr, 0, pt_ref.data() + i * L, L, want.data());
    CHECK(std::memcmp(ct + i * sct, want.data(), L + 16) == 0, "encrypt L=%u rec %llu %s", L,
          (unsigned long long)i, inplace ? "in place" : "copy");
    for (uint64_t b = L + 16; b < sct; ++b)
      if (ct[i * sct + b] != (inplace ? 0xA5 : 0x5A)) {
        CHECK(false, "encrypt L=%u rec %llu wrote gap byte %llu", L, (unsigned long long)i, (unsigned long long)b);
        break;
      }
  }
  // tamper: the tag's last byte, the first and the last ciphertext byte
  std::vector<uint8_t> bad(R, 0);
  for (uint64_t i = 0; i < R; i += 5) {
    const uint64_t pos = (i / 5) % 3 == 0 ? L + 15 : (i / 5) % 3 == 1 ? 0 : L - 1;
    ct[i * sct + pos] ^= 0x40;
    bad[i] = 1;
  }
  std::vector<uint8_t> ct_copy(ct, ct + R * sct);
  uint8_t *back = inplace ? ct : (uint8_t *)std::aligned_alloc(16, R * sin);
  if (!inplace) std::memset(back, 0xC3, R * sin);
  uint8_t *st = (uint8_t *)std::malloc(R);
  std::memset(st, 9, R);
  g_ext.clear();
  for (uint64_t i = 0; i < R; ++i)
    g_ext.push_back(Ext{reinterpret_cast<uintptr_t>(back + i * sin), reinterpret_cast<uintptr_t>(back + i * sin) + L, bad[i] != 0});
  g_inplace = inplace;
  emu::store_hook = watch;
  e = noise_amd::launch_aead_uniform(true, k, nonce0, ct, sct, back, sin, L, nullptr, 0, 0, st, R, nullptr);
  emu::store_hook = nullptr;
  CHECK(e == hipSuccess, "decrypt launch L=%u", L);
  for (uint64_t i = 0; i < R; ++i) {
    if (bad[i]) {
      CHECK(st[i] == 1, "status of tampered L=%u rec %llu = %u", L, (unsigned long long)i, st[i]);
      if (inplace)
        CHECK(std::memcmp(back + i * sin, ct_copy.data() + i * sct, L + 16) == 0, "in-place failure modified L=%u rec %llu",
              L, (unsigned long long)i);
      else
        for (uint32_t b = 0; b < L; ++b)
          if (back[i * sin + b] != 0) {
            CHECK(false, "failed copy not zeroed L=%u rec %llu", L, (unsigned long long)i);
            break;
          }
    } else {
      CHECK(st[i] == 0, "status L=%u rec %llu = %u", L, (unsigned long long)i, st[i]);
      CHECK(std::memcmp(back + i * sin, pt_ref.data() + i * L, L) == 0, "decrypt L=%u rec %llu %s", L,
            (unsigned long long)i, inplace ? "in place" : "copy");
    }
    if (inplace) {  // the tag bytes after the plaintext stay as they were
      CHECK(std::memcmp(back + i * sin + L, ct_copy.data() + i * sct + L, 16) == 0, "in-place decrypt wrote the tag L=%u", L);
    } else {
      for (uint64_t b = L; b < sin; ++b)
        if (back[i * sin + b] != 0xC3) {
          CHECK(false, "decrypt L=%u rec %llu wrote gap byte %llu", L, (unsigned long long)i, (unsigned long long)b);
          break;
        }
    }
  }
  std::free(st);
  if (!inplace) {
    std::free(ct);
    std::free(back);
  }
  std::free(pt);
}

// Unaligned records (strides and bases off 16; aead_kernels.hip stages them
// through an aligned scratch image): the oracle on every record, canary bytes
// between records untouched, tampered records fail (in place: untouched,
// copy: zeros).  No store watch: the tile kernels write the scratch image.
static void run_unaligned(uint32_t L, uint64_t seed, bool inplace, uint64_t R) {
  const uint64_t sin = inplace ? L + 16 + 3 : L + 3, sct = inplace ? sin : L + 16 + 5;
  const uint64_t oin = inplace ? 5 : 1, oct = inplace ? 5 : 7;
  uint8_t key[32];
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(mix64(seed + i) | 1);
  uint32_t k[8];
  std::memcpy(k, key, 32);
  const uint64_t nonce0 = mix64(seed * 3 + L) & 0xffffffffull;
  std::vector<uint8_t> pt_ref(R * L);
  for (uint64_t j = 0; j < R * L; ++j) pt_ref[j] = (uint8_t)mix64(seed * 17 + j);
  const uint64_t nbin = oin + R * sin + 16, nbct = oct + R * sct + 16;
  uint8_t *bin = (uint8_t *)std::aligned_alloc(16, (nbin + 15) / 16 * 16);
  uint8_t *bct = inplace ? bin : (uint8_t *)std::aligned_alloc(16, (nbct + 15) / 16 * 16);
  std::memset(bin, 0xA5, (nbin + 15) / 16 * 16);
  if (!inplace) std::memset(bct, 0x5A, (nbct + 15) / 16 * 16);
  uint8_t *pt = bin + oin, *ct = bct + oct;
  for (uint64_t i = 0; i < R; ++i) std::memcpy(pt + i * sin, pt_ref.data() + i * L, L);
  hipError_t e = noise_amd::launch_aead_uniform(false, k, nonce0, pt, sin, ct, sct, L, nullptr, 0, 0, nullptr, R, nullptr);
  CHECK(e == hipSuccess, "unaligned encrypt launch L=%u", L);
  std::vector<uint8_t> want(L + 16);
  const uint8_t fill = inplace ? 0xA5 : 0x5A;
  for (uint64_t i = 0; i < R; ++i) {
    oracle_noise_encrypt(key, nonce0 + i, nullptr, 0, pt_ref.data() + i * L, L, want.data());
    CHECK(std::memcmp(ct + i * sct, want.data(), L + 16) == 0, "unaligned encrypt L=%u rec %llu %s", L,
          (unsigned long long)i, inplace ? "in place" : "copy");
    for (uint64_t b = L + 16; b < sct; ++b)
      if (ct[i * sct + b] != fill) {
        CHECK(false, "unaligned encrypt L=%u rec %llu wrote gap byte %llu", L, (unsigned long long)i,
              (unsigned long long)b);
        break;
      }
  }
  if (!inplace) CHECK(bct[0] == fill && bct[oct - 1] == fill, "unaligned encrypt wrote before the first record");
  std::vector<uint8_t> bad(R, 0);
  for (uint64_t i = 3; i < R; i += 97) {
    const uint64_t pos = (i / 97) % 3 == 0 ? L + 15 : (i / 97) % 3 == 1 ? 0 : L - 1;
    ct[i * sct + pos] ^= 0x40;
    bad[i] = 1;
  }
  std::vector<uint8_t> ct_copy(ct, ct + R * sct);
  uint8_t *bback = inplace ? bct : (uint8_t *)std::aligned_alloc(16, (nbin + 15) / 16 * 16);
  if (!inplace) std::memset(bback, 0xC3, (nbin + 15) / 16 * 16);
  uint8_t *back = inplace ? ct : bback + oin;
  const uint64_t sb = inplace ? sct : sin;
  uint8_t *st = (uint8_t *)std::malloc(R);
  std::memset(st, 9, R);
  e = noise_amd::launch_aead_uniform(true, k, nonce0, ct, sct, back, sb, L, nullptr, 0, 0, st, R, nullptr);
  CHECK(e == hipSuccess, "unaligned decrypt launch L=%u", L);
  for (uint64_t i = 0; i < R; ++i) {
    if (bad[i]) {
      CHECK(st[i] == 1, "unaligned status of tampered L=%u rec %llu = %u", L, (unsigned long long)i, st[i]);
      if (inplace) {
        CHECK(std::memcmp(back + i * sb, ct_copy.data() + i * sct, L + 16) == 0, "unaligned in-place failure modified L=%u", L);
      } else {
        for (uint32_t b = 0; b < L; ++b)
          if (back[i * sb + b] != 0) {
            CHECK(false, "unaligned failed copy not zeroed L=%u rec %llu", L, (unsigned long long)i);
            break;
          }
      }
    } else {
      CHECK(st[i] == 0, "unaligned status L=%u rec %llu = %u", L, (unsigned long long)i, st[i]);
      CHECK(std::memcmp(back + i * sb, pt_ref.data() + i * L, L) == 0, "unaligned decrypt L=%u rec %llu %s", L,
            (unsigned long long)i, inplace ? "in place" : "copy");
    }
    if (inplace) {
      CHECK(std::memcmp(back + i * sb + L, ct_copy.data() + i * sct + L, 16) == 0, "unaligned in-place decrypt wrote the tag L=%u", L);
    } else {
      for (uint64_t b = L; b < sb; ++b)
        if (back[i * sb + b] != 0xC3) {
          CHECK(false, "unaligned decrypt L=%u rec %llu wrote gap byte %llu", L, (unsigned long long)i, (unsigned long long)b);
          break;
        }
    }
  }
  std::free(st);
  if (!inplace) {
    std::free(bct);
    std::free(bback);
  }
  std::free(bin);
}

int main(int argc, char **argv) {
  if (argc > 1 && std::strcmp(argv[1], "unaligned") == 0) {
    // records >= kStageMin (1024) take the staged path
    std::vector<uint32_t> lens = {1, 17, 100, 1000, 1023, 1040, 3000, 5000};
    if (argc > 2) {
      lens.clear();
      for (int i = 2; i < argc; ++i) lens.push_back((uint32_t)std::strtoul(argv[i], nullptr, 0));
    }
    for (uint32_t L : lens) {
      const uint64_t R = L > 2048 ? 1030 : 1100;
      run_unaligned(L, 11 + L, false, R);
      run_unaligned(L, 13 + L, true, R);
      std::printf("unaligned L=%u R=%llu ok so far (%d failures)\n", L, (unsigned long long)R, fails);
      std::fflush(stdout);
    }
    noise_amd::records_scratch_release(nullptr);  // the staging scratch
    std::printf("%s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
  }
  const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 3;
  std::vector<uint32_t> lens;
  for (int i = 2; i < argc; ++i) lens.push_back((uint32_t)std::strtoul(argv[i], nullptr, 0));
  if (lens.empty())
    lens = {1, 15, 16, 17, 33, 63, 65, 100, 127, 129, 191, 193, 255, 257, 300, 321, 384, 400, 449, 511, 513,
            700, 769, 1000, 1023, 1025, 1040, 1281, 1400, 1537, 1793, 2047, 2049, 2305, 2561, 3000, 3073, 4095,
            4097, 5000, 5121, 8191, 9000, 16000, 16383};
  for (uint32_t L : lens) {
    // a few tiles and a partial one (records per tile: 64 / max(1, L / 256))
    const uint64_t rpt = L >= 256 ? 64 / ((L + 255) / 256 > 64 ? 64 : (L + 255) / 256) : 64;  // ~ (capacity classes)
    const uint64_t R = L > 4096 ? 6 : rpt * 2 + 3;
    const long o0 = g_outside.load(), u0 = g_unverified.load();
    run(L, seed + L, false, R);
    run(L, seed + 7 * L, true, R);
    CHECK(g_outside.load() == o0, "L=%u: stores outside the records' outputs", L);
    CHECK(g_unverified.load() == u0, "L=%u: stores of unverified plaintext", L);
    std::printf("L=%u R=%llu ok so far (%d failures)\n", L, (unsigned long long)R, fails);
    std::fflush(stdout);
  }
  std::printf("uniform masked: %ld stores outside, %ld stores of unverified plaintext\n", g_outside.load(),
              g_unverified.load());
  std::printf("%s (%d failures)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
