// transport_test.cpp -- noise::transport (framing + multi-session batcher)
// against the CPU oracle (oracle/liboracle.so: test infrastructure).
//
//   transport_test <sessions> <messages> <seed>
// Sessions get random keys and start nonces; messages (0..2000 bytes, some
// 65519) are submitted interleaved, encrypted in ONE batch, checked bit-exact
// against oracle_noise_encrypt with each session's nonce sequence, framed per
// session into a byte stream, re-read through a Deframer fed in random-size
// chunks, decrypted in ONE batch (one record tampered per 97) and compared.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "noise_amd/transport.hpp"

extern "C" {
void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad, size_t ad_len,
                          const uint8_t *pt, size_t len, uint8_t *out);
}

using bytes = std::vector<std::uint8_t>;
namespace nt = noise::transport;

int main(int argc, char **argv) {
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
  std::printf("sessions %d messages %d: %s (%d failures)\n", S, M, fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
