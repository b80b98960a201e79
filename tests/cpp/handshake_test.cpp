// handshake_test.cpp -- drives noise::HandshakeState / SymmetricState
// (noise-cpp_amd/host/noise_amd/handshake.hpp) and the host primitives.
//
//   handshake_test blake2b <hex>             BLAKE2b-512 of the bytes
//   handshake_test hmac <keyhex> <hex>       HMAC-BLAKE2b
//   handshake_test hkdf <ckhex> <ikmhex>     Noise HKDF, 3 outputs
//   handshake_test x25519 <skhex> <uhex>     X25519
//   handshake_test patterns                  every enum pattern name, message count
//       (the above need no GPU: tests/test_handshake.py)
//   handshake_test vectors <tsv>             replay tests/golden/handshake_vectors.tsv
//       (handshake messages, handshake hash, transport records through the
//       GPU-backed CipherState; tests/test_gpu_parity.py, -m gpu)
//   handshake_test loopback <records> <len>  XX loopback handshake with fresh
//       keys + records each way (BASELINE config 1 shape), prints timings
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "noise_amd/handshake.hpp"

using bytes = std::vector<std::uint8_t>;

static bytes unhex(const std::string &s) {
  if (s == "-" ) return {};
  bytes b(s.size() / 2);
  for (std::size_t i = 0; i < b.size(); ++i) b[i] = (std::uint8_t)std::stoul(s.substr(2 * i, 2), nullptr, 16);
  return b;
}
static std::string hex(const std::uint8_t *p, std::size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s;
  for (std::size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}
template <class C> static std::string hex(const C &c) { return hex(c.data(), c.size()); }
static std::array<std::uint8_t, 32> a32(const std::string &s) {
  const bytes b = unhex(s);
  if (b.size() != 32) throw std::runtime_error("expected 32 bytes");
  std::array<std::uint8_t, 32> a;
  std::memcpy(a.data(), b.data(), 32);
  return a;
}
static std::vector<std::string> split(const std::string &s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  std::istringstream is(s);
  while (std::getline(is, cur, sep)) out.push_back(cur);
  if (!s.empty() && s.back() == sep) out.push_back("");
  return out;
}

struct Vec {
  std::string name, pattern;
  std::string f[11];  // FIELDS of make_handshake_vectors.py
  std::vector<std::pair<bytes, bytes>> msgs;
};

static noise::HandshakeStateConfiguration config(const Vec &v, bool init) {
  const int o = init ? 0 : 5;
  noise::HandshakeStateConfiguration c{};
  c.initiator = init;
  c.prologue = unhex(v.f[o + 0]);
  if (v.f[o + 1] != "-")
    for (const std::string &p : split(v.f[o + 1], ',')) c.psks.push_back(unhex(p));
  if (v.f[o + 2] != "-") c.s = noise::keypair_from_private(a32(v.f[o + 2]));
  if (v.f[o + 3] != "-") c.e = noise::keypair_from_private(a32(v.f[o + 3]));
  if (v.f[o + 4] != "-") c.rs = a32(v.f[o + 4]);
  return c;
}

static int run_vectors(const char *path) {
  std::ifstream in(path);
  if (!in) {
    std::printf("cannot open %s\n", path);
    return 2;
  }
  std::string line;
  int n = 0, fails = 0, transport = 0, hashes = 0;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    const std::vector<std::string> cols = split(line, '\t');
    if (cols.size() != 13) {
      std::printf("bad line\n");
      return 2;
    }
    Vec v;
    v.name = cols[0];
    v.pattern = split(v.name, '_')[1];
    for (int i = 0; i < 11; ++i) v.f[i] = cols[1 + i];
    for (const std::string &m : split(cols[12], ',')) {
      const std::size_t c = m.find(':');
      v.msgs.push_back({unhex(c == 0 ? "-" : m.substr(0, c)), unhex(m.substr(c + 1))});
    }
    ++n;
    try {
      noise::HandshakeState ini, res;
      ini.initialize_named(v.pattern, config(v, true));
      res.initialize_named(v.pattern, config(v, false));
      std::string base = v.pattern.substr(0, v.pattern.find("psk"));
      const bool one_way = base == "N" || base == "K" || base == "X";
      noise::CipherState i_send, i_recv, r_send, r_recv;
      bool done = false;
      for (std::size_t m = 0; m < v.msgs.size(); ++m) {
        const bool init_sends = one_way || (m % 2 == 0);
        bytes payload = v.msgs[m].first;
        const bytes &want = v.msgs[m].second;
        if (!done) {
          noise::HandshakeState &w = init_sends ? ini : res, &r = init_sends ? res : ini;
          bytes wire, got;
          w.write_message(payload, wire);
          if (wire != want) throw std::runtime_error("handshake message " + std::to_string(m) + " differs");
          r.read_message(wire, got);
          if (got != v.msgs[m].first) throw std::runtime_error("handshake payload " + std::to_string(m) + " differs");
          if (ini.is_handshake_finished() != res.is_handshake_finished())
            throw std::runtime_error("parties disagree on completion");
          if (ini.is_handshake_finished()) {
            done = true;
            const auto hi = ini.get_handshake_hash(), hr = res.get_handshake_hash();
            if (hi != hr) throw std::runtime_error("handshake hashes differ");
            if (v.f[10] != "-") {
              if (hex(hi) != v.f[10]) throw std::runtime_error("handshake_hash differs");
              ++hashes;
            }
            std::tie(i_send, i_recv) = ini.finalize();
            std::tie(r_recv, r_send) = res.finalize();
          }
        } else {
          noise::CipherState &snd = init_sends ? i_send : r_send, &rcv = init_sends ? r_recv : i_recv;
          bytes msg = payload;
          snd.encrypt_with_ad(msg);
          if (msg != want) throw std::runtime_error("transport message " + std::to_string(m) + " differs");
          rcv.decrypt_with_ad(msg);
          if (msg != v.msgs[m].first) throw std::runtime_error("transport payload " + std::to_string(m) + " differs");
          ++transport;
        }
      }
      if (!done) throw std::runtime_error("handshake did not finish");
    } catch (const std::exception &e) {
      if (fails < 20) std::printf("FAIL %s: %s\n", v.name.c_str(), e.what());
      ++fails;
    }
  }
  std::printf("vectors %d, failed %d, handshake hashes checked %d, transport records %d: %s\n", n,
              fails, hashes, transport, fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}

// XX loopback with fresh keys, as examples/Noise_XX_25519_ChaChaPoly_Blake2b.cpp
// (26-71), then `records` transport records of `len` bytes each way.
static int loopback(int records, int len, bool timed = true) {
  using clk = std::chrono::steady_clock;
  if (timed) loopback(4, 64, false);  // warm: device init, staging buffers
  const auto t0 = clk::now();
  noise::HandshakeStateConfiguration ci{}, cr{};
  ci.pattern = cr.pattern = noise::HandshakePattern::XX;
  ci.initiator = true;
  cr.initiator = false;
  ci.s = noise::generate_keypair();
  cr.s = noise::generate_keypair();
  noise::HandshakeState ini, res;
  ini.initialize(ci);
  res.initialize(cr);
  noise::HandshakeState *w = &ini, *r = &res;
  while (!ini.is_handshake_finished()) {
    bytes msg, payload;
    w->write_message(msg);
    r->read_message(msg, payload);
    std::swap(w, r);
  }
  auto [i_send, i_recv] = ini.finalize();
  auto [r_recv, r_send] = res.finalize();
  const auto t1 = clk::now();
  std::vector<bytes> batch(records);
  for (int i = 0; i < records; ++i) {
    batch[i].resize(len);
    for (int j = 0; j < len; ++j) batch[i][j] = (std::uint8_t)(7 * j + 3 + i);
  }
  const std::vector<bytes> orig = batch;
  i_send.encrypt_batch(batch);
  r_recv.decrypt_batch(batch);
  const bool ok1 = batch == orig;
  r_send.encrypt_batch(batch);
  i_recv.decrypt_batch(batch);
  const bool ok2 = batch == orig;
  const auto t2 = clk::now();
  const double hs = std::chrono::duration<double>(t1 - t0).count();
  const double tr = std::chrono::duration<double>(t2 - t1).count();
  if (timed)
    std::printf("{\"handshake_ms\": %.3f, \"records\": %d, \"record_bytes\": %d, \"transport_ms\": %.3f, "
                "\"ok\": %s}\n", hs * 1e3, records, len, tr * 1e3, ok1 && ok2 ? "true" : "false");
  return ok1 && ok2 ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string cmd = argv[1];
  try {
    if (cmd == "blake2b" && argc == 3) {
      const bytes b = unhex(argv[2]);
      std::printf("%s\n", hex(noise::crypto::blake2b(b.data(), b.size())).c_str());
    } else if (cmd == "hmac" && argc == 4) {
      const bytes k = unhex(argv[2]), d = unhex(argv[3]);
      std::printf("%s\n", hex(noise::crypto::hmac(k.data(), k.size(), d.data(), d.size())).c_str());
    } else if (cmd == "hkdf" && argc == 4) {
      const bytes c = unhex(argv[2]), ikm = unhex(argv[3]);
      noise::crypto::Hash ck, o1, o2, o3;
      std::memcpy(ck.data(), c.data(), 64);
      noise::crypto::hkdf(ck, ikm.data(), ikm.size(), &o1, &o2, &o3);
      std::printf("%s %s %s\n", hex(o1).c_str(), hex(o2).c_str(), hex(o3).c_str());
    } else if (cmd == "x25519" && argc == 4) {
      std::printf("%s\n", hex(noise::crypto::x25519(a32(argv[2]), a32(argv[3]))).c_str());
    } else if (cmd == "patterns") {
      for (int p = 0; p <= (int)noise::HandshakePattern::IXpsk2; ++p)
        std::printf("%s\n", std::string(noise::pattern_name((noise::HandshakePattern)p)).c_str());
    } else if (cmd == "vectors" && argc == 3) {
      return run_vectors(argv[2]);
    } else if (cmd == "loopback" && argc == 4) {
      return loopback(std::atoi(argv[2]), std::atoi(argv[3]));
    } else {
      return 2;
    }
  } catch (const std::exception &e) {
    std::printf("error: %s\n", e.what());
    return 1;
  }
  return 0;
}
