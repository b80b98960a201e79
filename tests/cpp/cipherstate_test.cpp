// tests/cpp/cipherstate_test.cpp -- drives the drop-in noise::CipherState
// (noise-cpp_amd/host) exactly as the reference's callers do
// (SymmetricState::encrypt_and_hash with AD = h, noise.cpp:498-515;
// transport encrypt_with_ad / decrypt_with_ad after split(), examples/
// Noise_XX_25519_ChaChaPoly_Blake2b.cpp:58-75) and checks every result
// against the golden records derived from the reference's tests/vectors.
//
//   cipherstate_test --host-only            checks that need no GPU
//   cipherstate_test <golden_dir>           full GPU run (pytest -m gpu)
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <optional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "noise_amd/cipher_state.hpp"

static int failures = 0;
#define CHECK(cond, ...)                                 \
  do {                                                   \
    if (!(cond)) {                                       \
      ++failures;                                        \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                 \
      std::fprintf(stderr, "\n");                        \
    }                                                    \
  } while (0)

using Bytes = std::vector<std::uint8_t>;

static Bytes unhex(const std::string &h) {
  Bytes b(h.size() / 2);
  for (std::size_t i = 0; i < b.size(); ++i) b[i] = (std::uint8_t)std::stoul(h.substr(2 * i, 2), nullptr, 16);
  return b;
}
static std::array<std::uint8_t, 32> key32(const std::string &h) {
  std::array<std::uint8_t, 32> k{};
  Bytes b = unhex(h);
  std::memcpy(k.data(), b.data(), 32);
  return k;
}
static bool zero32(const std::array<std::uint8_t, 32> &k) {
  for (auto b : k)
    if (b) return false;
  return true;
}
static std::vector<std::vector<std::string>> read_tsv(const std::string &path) {
  std::vector<std::vector<std::string>> rows;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::vector<std::string> cols;
    std::stringstream ss(line);
    std::string c;
    while (std::getline(ss, c, '\t')) cols.push_back(c);
    rows.push_back(cols);
  }
  return rows;
}

// ---- checks that never reach the device ----------------------------------
static void host_only_checks() {
  using noise::CipherState;
  {  // all-zero key == no key: encrypt/decrypt are pass-throughs (spec)
    CipherState cs;
    cs.initialize_key(std::array<std::uint8_t, 32>{});
    CHECK(!cs.has_key(), "zero key must read as no key");
    Bytes m = {1, 2, 3};
    cs.encrypt_with_ad(m);
    CHECK(m == Bytes({1, 2, 3}), "no-key encrypt must not change the message");
    cs.decrypt_with_ad(m);
    CHECK(m == Bytes({1, 2, 3}), "no-key decrypt must not change the message");
    CHECK(cs.nonce() == 0, "no-key calls must not advance n");
  }
  {  // nonce limit: n == 2^64-2 throws out_of_range before any device work
    CipherState cs;
    std::array<std::uint8_t, 32> k{};
    k[0] = 1;
    cs.initialize_key(k);
    CHECK(cs.has_key(), "non-zero key must read as a key");
    cs.set_nonce(std::numeric_limits<std::uint64_t>::max() - 1);
    Bytes m = {9};
    bool threw = false;
    try { cs.encrypt_with_ad(m); } catch (const std::out_of_range &e) {
      threw = std::string(e.what()) == "Nonce limit has been exceeded!";
    }
    CHECK(threw, "encrypt at n = 2^64-2 must throw out_of_range");
    CHECK(m == Bytes({9}), "refused encrypt must not touch the message");
    threw = false;
    try { cs.decrypt_with_ad(m); } catch (const std::out_of_range &) { threw = true; }
    CHECK(threw, "decrypt at n = 2^64-2 must throw out_of_range");
    CHECK(cs.nonce() == std::numeric_limits<std::uint64_t>::max() - 1, "n unchanged");
    // batch at the limit: nothing processed, throws
    std::vector<Bytes> batch = {{1}, {2}};
    threw = false;
    try { cs.encrypt_batch(batch); } catch (const std::out_of_range &) { threw = true; }
    CHECK(threw && batch[0] == Bytes({1}), "batch at the limit must throw untouched");
  }
  {  // layout is the reference's: 32-byte key + 64-bit nonce
    static_assert(sizeof(noise::CipherState) == 40, "CipherState layout must match noise.h");
  }
}

// ---- GPU checks -----------------------------------------------------------
static void gpu_checks(const std::string &dir) {
  using noise::CipherState;
  // 1. transport records: encrypt_with_ad(pt) at (k, n) == golden ct||tag
  auto tr = read_tsv(dir + "/transport_records.tsv");
  CHECK(tr.size() == 1688, "expected 1688 transport records, got %zu", tr.size());
  int n_ok = 0;
  for (auto &r : tr) {
    CipherState cs;
    cs.initialize_key(key32(r[2]));
    cs.set_nonce(std::stoull(r[3]));
    Bytes m = unhex(r[4]);
    const Bytes want = unhex(r[5]);
    cs.encrypt_with_ad(m);
    CHECK(m == want, "transport %s n=%s mismatch", r[0].c_str(), r[3].c_str());
    CipherState rx;
    rx.initialize_key(key32(r[2]));
    rx.set_nonce(std::stoull(r[3]));
    rx.decrypt_with_ad(m);
    CHECK(m == unhex(r[4]), "transport decrypt %s mismatch", r[0].c_str());
    n_ok += (m == unhex(r[4]));
  }
  // 2. handshake records: encrypt_with_ad(ad = h, pt), the SymmetricState path
  auto hs = read_tsv(dir + "/handshake_records.tsv");
  CHECK(hs.size() == 1828, "expected 1828 handshake records, got %zu", hs.size());
  for (auto &r : hs) {
    CipherState cs;
    cs.initialize_key(key32(r[1]));
    cs.set_nonce(std::stoull(r[2]));
    Bytes ad = unhex(r[3]), m = unhex(r[4]);
    cs.encrypt_with_ad(ad, m);
    CHECK(m == unhex(r[5]), "handshake %s n=%s mismatch", r[0].c_str(), r[2].c_str());
    CipherState rx;
    rx.initialize_key(key32(r[1]));
    rx.set_nonce(std::stoull(r[2]));
    rx.decrypt_with_ad(ad, m);
    CHECK(m == unhex(r[4]), "handshake decrypt %s mismatch", r[0].c_str());
  }
  // 3. sequential nonces and MAC failure semantics (n advances, buffer kept)
  {
    auto &r = tr[0];
    CipherState tx, rx;
    tx.initialize_key(key32(r[2]));
    rx.initialize_key(key32(r[2]));
    std::vector<Bytes> sent;
    for (int i = 0; i < 5; ++i) {
      Bytes m(17 * i + 3, (std::uint8_t)i);
      tx.encrypt_with_ad(m);
      sent.push_back(m);
    }
    CHECK(tx.nonce() == 5, "tx nonce after 5 records");
    Bytes bad = sent[0];
    bad[0] ^= 1;
    const Bytes bad_copy = bad;
    bool threw = false;
    try { rx.decrypt_with_ad(bad); } catch (const std::invalid_argument &e) {
      threw = std::string(e.what()) == "Invalid MAC";
    }
    CHECK(threw, "tampered record must throw invalid_argument(\"Invalid MAC\")");
    CHECK(bad == bad_copy, "failed decrypt must leave the buffer untouched");
    CHECK(rx.nonce() == 1, "n advances on MAC failure (noise.cpp:421)");
    for (int i = 1; i < 5; ++i) {
      Bytes m = sent[i];
      rx.decrypt_with_ad(m);
      CHECK(m == Bytes(17 * i + 3, (std::uint8_t)i), "record %d round trip", i);
    }
    Bytes tiny = {1, 2, 3};
    threw = false;
    try { rx.decrypt_with_ad(tiny); } catch (const std::invalid_argument &) { threw = true; }
    CHECK(threw, "ciphertext shorter than the tag must throw invalid_argument");
  }
  // 4. rekey KAT: rekey of the all-zero key
  {
    CipherState cs;
    cs.initialize_key(std::array<std::uint8_t, 32>{});
    cs.rekey();
    CHECK(cs.has_key(), "rekeyed zero key is a key");
    // the new key must encrypt like key K4
    CipherState ref;
    ref.initialize_key(key32("765f5f43857ccfe16f686cb1f02213efb5cad57191351e67b517961142410e93"));
    Bytes a = {1, 2, 3, 4}, b = a;
    cs.encrypt_with_ad(a);
    ref.encrypt_with_ad(b);
    CHECK(a == b, "rekey(0^32) must equal K4");
  }
  // 5. n = 2^64-1 is accepted (then wraps to 0), as in the reference
  {
    CipherState cs;
    cs.initialize_key(key32(tr[0][2]));
    cs.set_nonce(std::numeric_limits<std::uint64_t>::max());
    Bytes m = {7, 7};
    cs.encrypt_with_ad(m);
    CHECK(m.size() == 18 && cs.nonce() == 0, "encrypt at 2^64-1 wraps n to 0");
  }
  // 6. batch API == per-record API (mixed lengths), including failures
  {
    auto k = key32(tr[5][2]);
    CipherState a, b;
    a.initialize_key(k);
    b.initialize_key(k);
    std::vector<Bytes> batch;
    for (int i = 0; i < 40; ++i) batch.push_back(Bytes((i * 37) % 300, (std::uint8_t)(i * 5)));
    std::vector<Bytes> single = batch;
    a.encrypt_batch(batch);
    for (auto &m : single) b.encrypt_with_ad(m);
    CHECK(batch == single && a.nonce() == b.nonce(), "encrypt_batch == encrypt_with_ad loop");
    CipherState rx;
    rx.initialize_key(k);
    batch[3][0] ^= 0x80;
    std::vector<std::uint8_t> ok;
    bool threw = false;
    try { rx.decrypt_batch(batch, &ok); } catch (const std::invalid_argument &) { threw = true; }
    CHECK(threw && ok.size() == 40 && !ok[3] && ok[4] && rx.nonce() == 40,
          "decrypt_batch flags the tampered record, advances n for all");
    CHECK(batch[4] == Bytes((4 * 37) % 300, (std::uint8_t)20), "good records decrypted");
    // batch crossing the nonce limit: records before it processed, then throw
    CipherState lim;
    lim.initialize_key(k);
    lim.set_nonce(std::numeric_limits<std::uint64_t>::max() - 3);
    std::vector<Bytes> four = {{1}, {2}, {3}, {4}};
    threw = false;
    try { lim.encrypt_batch(four); } catch (const std::out_of_range &) { threw = true; }
    CHECK(threw && four[0].size() == 17 && four[1].size() == 17 && four[2].size() == 1,
          "batch stops at the nonce limit after 2 records");
    CHECK(lim.nonce() == std::numeric_limits<std::uint64_t>::max() - 1, "n at the limit");
  }
  // 7. the reference's free functions noise::encrypt / noise::decrypt
  // (noise.cpp:202-224, 254-281) over every golden record: same bytes, the
  // caller's key wiped after each call, resize +-16, Invalid MAC on a tamper
  // with the buffer untouched
  {
    int nf = 0;
    for (auto &r : tr) {
      auto k = key32(r[2]);
      Bytes m = unhex(r[4]);
      noise::encrypt(k, std::stoull(r[3]), std::nullopt, m);
      CHECK(m == unhex(r[5]), "free encrypt %s n=%s", r[0].c_str(), r[3].c_str());
      CHECK(zero32(k), "free encrypt must wipe the key (noise.cpp:222)");
      k = key32(r[2]);
      noise::decrypt(k, std::stoull(r[3]), std::nullopt, m);
      CHECK(m == unhex(r[4]), "free decrypt %s", r[0].c_str());
      CHECK(zero32(k), "free decrypt must wipe the key");
      nf += m == unhex(r[4]);
    }
    for (auto &r : hs) {
      auto k = key32(r[1]);
      Bytes m = unhex(r[4]);
      const std::optional<Bytes> ad = unhex(r[3]);
      noise::encrypt(k, std::stoull(r[2]), ad, m);
      CHECK(m == unhex(r[5]), "free encrypt (AD) %s n=%s", r[0].c_str(), r[2].c_str());
      k = key32(r[1]);
      noise::decrypt(k, std::stoull(r[2]), ad, m);
      CHECK(m == unhex(r[4]), "free decrypt (AD) %s", r[0].c_str());
      nf += m == unhex(r[4]);
    }
    auto k = key32(tr[0][2]);
    Bytes m = unhex(tr[0][5]);
    m[m.size() - 1] ^= 1;
    const Bytes before = m;
    bool threw = false;
    try { noise::decrypt(k, std::stoull(tr[0][3]), std::nullopt, m); } catch (const std::invalid_argument &e) {
      threw = std::string(e.what()) == "Invalid MAC";
    }
    CHECK(threw && m == before, "tampered free decrypt: Invalid MAC, buffer untouched");
    CHECK(zero32(k), "failed free decrypt still wipes the key (noise.cpp:272)");
    k = key32(tr[0][2]);
    Bytes tiny = {1, 2};
    threw = false;
    try { noise::decrypt(k, 0, std::nullopt, tiny); } catch (const std::invalid_argument &) { threw = true; }
    CHECK(threw && tiny.size() == 2, "free decrypt of < 16 bytes throws (reference: underflow)");
    std::printf("free functions: %d/%zu golden round trips ok\n", nf, tr.size() + hs.size());
  }
  std::printf("transport %d/%zu round trips ok\n", n_ok, tr.size());
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s --host-only | <golden_dir>\n", argv[0]);
    return 2;
  }
  host_only_checks();
  if (std::string(argv[1]) != "--host-only") {
    try {
      gpu_checks(argv[1]);
    } catch (const std::exception &e) {
      std::fprintf(stderr, "FAIL: exception %s\n", e.what());
      ++failures;
    }
  }
  std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED", failures);
  return failures ? 1 : 0;
}
