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
//   handshake_test batch_vectors <tsv>       the same vectors through the
//       batched GPU handshake (noise_gpu_hs_*): all vectors of a pattern in
//       one batch per role; messages, handshake hashes, split keys (the
//       transport records through CipherStates keyed by them)
//   handshake_test batch_check <pattern> <n> <seed>  n sessions of a pattern
//       through the batched GPU handshake with preset keys and random
//       payloads vs the host HandshateState per session (every message), plus
//       tampered messages failing exactly their sessions
//   handshake_test batch_bench <pattern> <n> <reps>  full handshakes/s of
//       the batched GPU handshake (fresh DRBG ephemerals, empty payloads)
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include <map>
#include <random>

#include "noise_amd/handshake.hpp"
#include "noise_gpu.h"

using bytes = std::vector<std::uint8_t>;
using noise::PatternToken;

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

// ---- batched GPU handshakes (noise_gpu_hs_*) ------------------------------
#define HIPCHK(x)                                                               \
  do {                                                                          \
    if ((x) != hipSuccess) throw std::runtime_error(std::string("HIP: ") + #x); \
  } while (0)
#define HSCHK(x)                                                                          \
  do {                                                                                    \
    const int rc_ = (x);                                                                  \
    if (rc_) throw std::runtime_error(std::string(#x) + ": " + noise_gpu_last_error()); \
  } while (0)

struct Dev {
  std::uint8_t *p = nullptr;
  std::size_t n = 0;
  explicit Dev(std::size_t bytes) : n(bytes) { HIPCHK(hipMalloc(&p, bytes ? bytes : 16)); HIPCHK(hipMemset(p, 0, bytes ? bytes : 16)); }
  ~Dev() { (void)hipFree(p); }
  Dev(const Dev &) = delete;
  void put(const void *h, std::size_t bytes) { HIPCHK(hipMemcpy(p, h, bytes, hipMemcpyHostToDevice)); }
  void get(void *h, std::size_t bytes) const { HIPCHK(hipMemcpy(h, p, bytes, hipMemcpyDeviceToHost)); }
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// Ragged per-session buffers packed at 16-byte aligned offsets on the device
struct Ragged {
  std::vector<std::uint64_t> off;
  std::vector<std::uint32_t> len;
  std::unique_ptr<Dev> data, doff, dlen;
  Ragged(const std::vector<bytes> &items, std::size_t room) {
    std::uint64_t o = 0;
    for (const bytes &b : items) {
      off.push_back(o);
      len.push_back((std::uint32_t)b.size());
      o += (b.size() + room + 15) & ~std::size_t(15);
    }
    data = std::make_unique<Dev>(o);
    std::vector<std::uint8_t> h(o ? o : 1, 0);
    for (std::size_t i = 0; i < items.size(); ++i)
      if (!items[i].empty()) std::memcpy(h.data() + off[i], items[i].data(), items[i].size());
    data->put(h.data(), o);
    doff = std::make_unique<Dev>(off.size() * 8);
    doff->put(off.data(), off.size() * 8);
    dlen = std::make_unique<Dev>(len.size() * 4);
    dlen->put(len.data(), len.size() * 4);
  }
  noise_gpu_span span() const {
    noise_gpu_span s{};
    s.base = data->p;
    s.off = doff->as<std::uint64_t>();
    s.len = dlen->as<std::uint32_t>();
    return s;
  }
  bytes item(std::size_t i, std::uint32_t n) const {
    bytes b(n);
    if (n) HIPCHK(hipMemcpy(b.data(), data->p + off[i], n, hipMemcpyDeviceToHost));
    return b;
  }
};

struct BatchSide {
  noise_gpu_hs *hs = nullptr;
  ~BatchSide() { noise_gpu_hs_destroy(hs); }
};

// per-session key material of one role (absent: empty)
struct RoleKeys {
  std::vector<bytes> prologue, s, e, rs;
  std::vector<std::vector<bytes>> psks;
};

static void set_role(BatchSide &b, const std::string &pattern, bool init, const RoleKeys &k,
                     std::size_t n) {
  HSCHK(noise_gpu_hs_create(pattern.c_str(), init, n, &b.hs));
  auto put_keys = [&](int slot, const std::vector<bytes> &v) {
    if (v.empty() || v[0].empty()) return;
    Dev d(32 * n);
    bytes all;
    for (const bytes &x : v) all.insert(all.end(), x.begin(), x.end());
    d.put(all.data(), all.size());
    HSCHK(noise_gpu_hs_set_key(b.hs, slot, d.p, 32, nullptr));
    HIPCHK(hipDeviceSynchronize());
  };
  put_keys(NOISE_GPU_HS_S, k.s);
  put_keys(NOISE_GPU_HS_E, k.e);
  put_keys(NOISE_GPU_HS_RS, k.rs);
  if (!k.psks.empty() && !k.psks[0].empty()) {
    bytes all;
    for (const auto &v : k.psks)
      for (const bytes &x : v) all.insert(all.end(), x.begin(), x.end());
    Dev d(all.size());
    d.put(all.data(), all.size());
    HSCHK(noise_gpu_hs_set_psks(b.hs, d.p, nullptr));
    HIPCHK(hipDeviceSynchronize());
  }
  Ragged pro(k.prologue, 0);
  noise_gpu_span ps = pro.span();
  HSCHK(noise_gpu_hs_start(b.hs, &ps, nullptr));
  HIPCHK(hipDeviceSynchronize());
}

// One handshake message from `w` to `r` for all sessions: returns the wire
// messages; received payloads and per-session status into *got / *status.
static std::vector<bytes> batch_message(BatchSide &w, BatchSide &r, const std::vector<bytes> &payloads,
                                        std::vector<bytes> *got, std::vector<std::uint8_t> *status,
                                        const std::vector<std::pair<std::size_t, std::size_t>> &tamper = {}) {
  const std::size_t n = payloads.size();
  noise_gpu_hs_info info;
  HSCHK(noise_gpu_hs_info_get(w.hs, &info));
  Ragged pay(payloads, 0);
  Ragged msg(payloads, info.overhead);
  Dev mlen(4 * n);
  noise_gpu_span ps = pay.span(), ms = msg.span();
  HSCHK(noise_gpu_hs_write_message(w.hs, &ps, &ms, mlen.as<std::uint32_t>(), nullptr));
  HIPCHK(hipDeviceSynchronize());
  std::vector<std::uint32_t> ml(n);
  mlen.get(ml.data(), 4 * n);
  std::vector<bytes> wire(n);
  for (std::size_t i = 0; i < n; ++i) {
    if (ml[i] != info.overhead + payloads[i].size()) throw std::runtime_error("message length");
    wire[i] = msg.item(i, ml[i]);
  }
  for (auto [i, byte] : tamper) {  // flip one bit of session i's message
    std::uint8_t v;
    HIPCHK(hipMemcpy(&v, msg.data->p + msg.off[i] + byte, 1, hipMemcpyDeviceToHost));
    v ^= 0x20;
    HIPCHK(hipMemcpy(msg.data->p + msg.off[i] + byte, &v, 1, hipMemcpyHostToDevice));
  }
  msg.dlen->put(ml.data(), 4 * n);
  Ragged out(payloads, 16);
  Dev plen(4 * n), st(n);
  noise_gpu_span ms2 = msg.span(), os = out.span();
  HSCHK(noise_gpu_hs_read_message(r.hs, &ms2, &os, plen.as<std::uint32_t>(), st.p, nullptr));
  HIPCHK(hipDeviceSynchronize());
  std::vector<std::uint32_t> pl(n);
  plen.get(pl.data(), 4 * n);
  status->resize(n);
  st.get(status->data(), n);
  got->resize(n);
  for (std::size_t i = 0; i < n; ++i) (*got)[i] = out.item(i, (*status)[i] ? 0 : pl[i]);
  return wire;
}

struct SplitOut {
  std::vector<std::array<std::uint8_t, 32>> k1, k2;
  std::vector<std::array<std::uint8_t, 64>> hash;
};
static SplitOut batch_split(BatchSide &b, std::size_t n) {
  Dev k1(32 * n), k2(32 * n), h(64 * n);
  HSCHK(noise_gpu_hs_split(b.hs, k1.p, k2.p, h.p, nullptr, nullptr));
  HIPCHK(hipDeviceSynchronize());
  SplitOut o;
  o.k1.resize(n);
  o.k2.resize(n);
  o.hash.resize(n);
  k1.get(o.k1.data(), 32 * n);
  k2.get(o.k2.data(), 32 * n);
  h.get(o.hash.data(), 64 * n);
  return o;
}

static int run_batch_vectors(const char *path) {
  std::ifstream in(path);
  if (!in) return 2;
  std::vector<Vec> all;
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    const std::vector<std::string> cols = split(line, '\t');
    Vec v;
    v.name = cols[0];
    v.pattern = split(v.name, '_')[1];
    for (int i = 0; i < 11; ++i) v.f[i] = cols[1 + i];
    for (const std::string &m : split(cols[12], ',')) {
      const std::size_t c = m.find(':');
      v.msgs.push_back({unhex(c == 0 ? "-" : m.substr(0, c)), unhex(m.substr(c + 1))});
    }
    all.push_back(v);
  }
  // one batch per (pattern, which keys are present, message count)
  std::map<std::string, std::vector<const Vec *>> groups;
  for (const Vec &v : all) {
    std::string key = v.pattern + "/" + std::to_string(v.msgs.size()) + "/";
    for (int i = 0; i < 11; ++i) key += v.f[i] == "-" ? '0' : '1';
    groups[key].push_back(&v);
  }
  int fails = 0, sessions = 0, batches = 0, transport = 0, hashes = 0;
  for (const auto &[key, vs] : groups) {
    const std::size_t n = vs.size();
    const std::string pattern = vs[0]->pattern;
    try {
      const noise::detail::PatternProgram prog = noise::detail::parse_pattern(pattern);
      RoleKeys ki, kr;
      for (const Vec *v : vs) {
        for (int side = 0; side < 2; ++side) {
          RoleKeys &k = side ? kr : ki;
          const int o = side ? 5 : 0;
          k.prologue.push_back(unhex(v->f[o]));
          std::vector<bytes> psk;
          if (v->f[o + 1] != "-")
            for (const std::string &p : split(v->f[o + 1], ',')) psk.push_back(unhex(p));
          k.psks.push_back(psk);
          k.s.push_back(unhex(v->f[o + 2]));
          k.e.push_back(unhex(v->f[o + 3]));
          k.rs.push_back(unhex(v->f[o + 4]));
        }
      }
      BatchSide ini, res;
      set_role(ini, pattern, true, ki, n);
      set_role(res, pattern, false, kr, n);
      const std::size_t nhs = prog.msgs.size();
      for (std::size_t m = 0; m < nhs; ++m) {
        const bool init_sends = prog.one_way || m % 2 == 0;
        std::vector<bytes> payloads(n), got;
        std::vector<std::uint8_t> st;
        for (std::size_t i = 0; i < n; ++i) payloads[i] = vs[i]->msgs[m].first;
        const std::vector<bytes> wire =
            batch_message(init_sends ? ini : res, init_sends ? res : ini, payloads, &got, &st);
        for (std::size_t i = 0; i < n; ++i) {
          if (wire[i] != vs[i]->msgs[m].second)
            throw std::runtime_error(vs[i]->name + ": message " + std::to_string(m) + " differs");
          if (st[i] != 0 || got[i] != payloads[i])
            throw std::runtime_error(vs[i]->name + ": payload " + std::to_string(m) + " not recovered");
        }
      }
      const SplitOut si = batch_split(ini, n), sr = batch_split(res, n);
      for (std::size_t i = 0; i < n; ++i) {
        const Vec &v = *vs[i];
        if (si.k1[i] != sr.k1[i] || si.k2[i] != sr.k2[i] || si.hash[i] != sr.hash[i])
          throw std::runtime_error(v.name + ": the two sides' split differs");
        if (v.f[10] != "-") {
          if (hex(si.hash[i]) != v.f[10]) throw std::runtime_error(v.name + ": handshake_hash differs");
          ++hashes;
        }
        noise::CipherState i_send, i_recv, r_send, r_recv;
        i_send.initialize_key(si.k1[i]);
        r_recv.initialize_key(sr.k1[i]);
        i_recv.initialize_key(si.k2[i]);
        r_send.initialize_key(sr.k2[i]);
        for (std::size_t m = nhs; m < v.msgs.size(); ++m) {
          const bool init_sends = prog.one_way || m % 2 == 0;
          noise::CipherState &snd = init_sends ? i_send : r_send, &rcv = init_sends ? r_recv : i_recv;
          bytes msg = v.msgs[m].first;
          snd.encrypt_with_ad(msg);
          if (msg != v.msgs[m].second) throw std::runtime_error(v.name + ": transport message differs");
          rcv.decrypt_with_ad(msg);
          if (msg != v.msgs[m].first) throw std::runtime_error(v.name + ": transport payload differs");
          ++transport;
        }
      }
      sessions += (int)n;
      ++batches;
    } catch (const std::exception &e) {
      if (fails < 20) std::printf("FAIL %s (%zu sessions): %s\n", key.c_str(), n, e.what());
      fails += (int)n;
    }
  }
  std::printf("batched vectors %d in %d batches, failed %d, handshake hashes checked %d, transport records %d: %s\n",
              sessions, batches, fails, hashes, transport, fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}

static bytes rand_bytes(std::mt19937_64 &g, std::size_t n) {
  bytes b(n);
  for (auto &x : b) x = (std::uint8_t)g();
  return b;
}

// n sessions of `pattern` with preset keys and random payloads on the GPU,
// every message and the handshake hash against the host HandshakeState of a
// sample of sessions, all sessions' split agreeing between the sides; then
// the same with tampered messages.
static int run_batch_check(const std::string &pattern, std::size_t n, unsigned seed) {
  std::mt19937_64 g(seed);
  const noise::detail::PatternProgram prog = noise::detail::parse_pattern(pattern);
  // which keys each side needs up front: statics always; rs when the peer's
  // static is a pre-message
  auto pre_has = [](const std::vector<PatternToken> &t, PatternToken x) {
    for (PatternToken y : t) if (y == x) return true;
    return false;
  };
  RoleKeys ki, kr;
  std::vector<noise::KeyPair> si(n), sr(n), ei(n), er(n);
  for (std::size_t i = 0; i < n; ++i) {
    std::array<std::uint8_t, 32> a;
    for (auto *kp : {&si[i], &sr[i], &ei[i], &er[i]}) {
      for (auto &x : a) x = (std::uint8_t)g();
      *kp = noise::keypair_from_private(a);
    }
    const bytes pro = rand_bytes(g, g() % 40);
    ki.prologue.push_back(pro);
    kr.prologue.push_back(pro);
    ki.s.emplace_back(si[i].sk.begin(), si[i].sk.end());
    kr.s.emplace_back(sr[i].sk.begin(), sr[i].sk.end());
    ki.e.emplace_back(ei[i].sk.begin(), ei[i].sk.end());
    kr.e.emplace_back(er[i].sk.begin(), er[i].sk.end());
    std::vector<bytes> psks;
    for (std::size_t p = 0; p < prog.npsk; ++p) psks.push_back(rand_bytes(g, 32));
    ki.psks.push_back(psks);
    kr.psks.push_back(psks);
    ki.rs.push_back(pre_has(prog.pre_r, PatternToken::S) ? bytes(sr[i].pk.begin(), sr[i].pk.end()) : bytes());
    kr.rs.push_back(pre_has(prog.pre_i, PatternToken::S) ? bytes(si[i].pk.begin(), si[i].pk.end()) : bytes());
  }
  // host reference for a sample of sessions
  const std::size_t nsample = std::min<std::size_t>(n, 24);
  std::vector<std::size_t> sample;
  for (std::size_t j = 0; j < nsample; ++j) sample.push_back(j == 0 ? 0 : j == 1 ? n - 1 : g() % n);
  std::vector<std::unique_ptr<noise::HandshakeState>> hi(nsample), hr(nsample);
  for (std::size_t j = 0; j < nsample; ++j) {
    const std::size_t i = sample[j];
    noise::HandshakeStateConfiguration ci{}, cr{};
    ci.initiator = true;
    cr.initiator = false;
    ci.prologue = ki.prologue[i];
    cr.prologue = kr.prologue[i];
    ci.s = si[i];
    cr.s = sr[i];
    ci.e = ei[i];
    cr.e = er[i];
    if (!ki.rs[i].empty()) ci.rs = sr[i].pk;
    if (!kr.rs[i].empty()) cr.rs = si[i].pk;
    ci.psks = ki.psks[i];
    cr.psks = kr.psks[i];
    hi[j] = std::make_unique<noise::HandshakeState>();
    hr[j] = std::make_unique<noise::HandshakeState>();
    hi[j]->initialize_named(pattern, ci);
    hr[j]->initialize_named(pattern, cr);
  }
  BatchSide bi, br;
  set_role(bi, pattern, true, ki, n);
  set_role(br, pattern, false, kr, n);
  std::size_t checked = 0;
  for (std::size_t m = 0; m < prog.msgs.size(); ++m) {
    const bool init_sends = prog.one_way || m % 2 == 0;
    std::vector<bytes> payloads(n), got;
    for (auto &p : payloads) p = rand_bytes(g, g() % 3 == 0 ? 0 : g() % 200);
    std::vector<std::uint8_t> st;
    const std::vector<bytes> wire =
        batch_message(init_sends ? bi : br, init_sends ? br : bi, payloads, &got, &st);
    for (std::size_t i = 0; i < n; ++i)
      if (st[i] || got[i] != payloads[i]) throw std::runtime_error("payload not recovered, session " + std::to_string(i));
    for (std::size_t j = 0; j < nsample; ++j) {
      const std::size_t i = sample[j];
      noise::HandshakeState &w = init_sends ? *hi[j] : *hr[j], &r = init_sends ? *hr[j] : *hi[j];
      bytes p = payloads[i], out, back;
      w.write_message(p, out);
      if (out != wire[i]) throw std::runtime_error("message " + std::to_string(m) + " differs from the host, session " + std::to_string(i));
      r.read_message(out, back);
      ++checked;
    }
  }
  const SplitOut oi = batch_split(bi, n), orr = batch_split(br, n);
  for (std::size_t i = 0; i < n; ++i)
    if (oi.k1[i] != orr.k1[i] || oi.k2[i] != orr.k2[i] || oi.hash[i] != orr.hash[i])
      throw std::runtime_error("sides disagree, session " + std::to_string(i));
  for (std::size_t j = 0; j < nsample; ++j) {
    const std::size_t i = sample[j];
    if (hi[j]->get_handshake_hash() != oi.hash[i]) throw std::runtime_error("handshake hash differs from the host");
    auto [c1, c2] = hi[j]->finalize();
    bytes a(64, 7), b = a;
    c1.encrypt_with_ad(a);
    noise::CipherState g1;
    g1.initialize_key(oi.k1[i]);
    g1.encrypt_with_ad(b);
    if (a != b) throw std::runtime_error("split key k1 differs from the host");
  }
  // tampering: a bit flip in the last message of sessions 0 and n/2 (for a
  // pattern whose last message carries a tag) fails exactly those sessions
  std::size_t tampered = 0;
  {
    BatchSide ti, tr;
    set_role(ti, pattern, true, ki, n);
    set_role(tr, pattern, false, kr, n);
    for (std::size_t m = 0; m < prog.msgs.size(); ++m) {
      const bool init_sends = prog.one_way || m % 2 == 0;
      std::vector<bytes> payloads(n, bytes(5, 1)), got;
      std::vector<std::uint8_t> st;
      noise_gpu_hs_info info;
      HSCHK(noise_gpu_hs_info_get(init_sends ? ti.hs : tr.hs, &info));
      std::vector<std::pair<std::size_t, std::size_t>> flips;
      const bool last = m + 1 == prog.msgs.size();
      if (last) flips = {{0, info.overhead + 4}, {n / 2, 0}};
      batch_message(init_sends ? ti : tr, init_sends ? tr : ti, payloads, &got, &st, flips);
      if (last) {
        for (std::size_t i = 0; i < n; ++i) {
          const bool hit = i == 0 || i == n / 2;
          if (hit && st[i] != NOISE_GPU_HS_BAD_MAC) throw std::runtime_error("tampered session not rejected");
          if (!hit && st[i] != 0) throw std::runtime_error("untampered session rejected");
          tampered += hit;
        }
      }
    }
    const std::size_t lastm = prog.msgs.size() - 1;
    const SplitOut z = batch_split(prog.one_way || lastm % 2 == 0 ? tr : ti, n);
    std::array<std::uint8_t, 32> zero{};
    if (z.k1[0] != zero) throw std::runtime_error("failed session got keys");
    if (n > 2 && z.k1[1] == zero) throw std::runtime_error("good session got zero keys");
  }
  std::printf("batch_check %s n=%zu: %zu host-checked messages, %zu tampered sessions rejected: ok\n",
              pattern.c_str(), n, checked, tampered);
  return 0;
}

// Full handshakes/s: both roles of `pattern` for n sessions, fresh DRBG
// ephemerals, empty payloads, random statics (one per side, stride 0: a
// server key and a client key), all on one stream.
static int run_batch_bench(const std::string &pattern, std::size_t n, int reps) {
  const noise::detail::PatternProgram prog = noise::detail::parse_pattern(pattern);
  const noise::KeyPair a = noise::generate_keypair(), b = noise::generate_keypair();
  Dev sa(32), sb(32), pa(32), pb(32);
  sa.put(a.sk.data(), 32);
  sb.put(b.sk.data(), 32);
  pa.put(a.pk.data(), 32);
  pb.put(b.pk.data(), 32);
  Dev psk(32 * n * (prog.npsk ? prog.npsk : 1));
  const std::size_t cap = 128;  // message stride: any overhead is <= 32 + 48 + 16
  Dev msg(cap * n), mlen(4 * n), st(n), k1(32 * n), k2(32 * n);
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  double best = 1e30;
  for (int r = 0; r < reps + 1; ++r) {
    BatchSide ini, res;  // allocation outside the timed region
    HSCHK(noise_gpu_hs_create(pattern.c_str(), 1, n, &ini.hs));
    HSCHK(noise_gpu_hs_create(pattern.c_str(), 0, n, &res.hs));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipEventRecord(e0, nullptr));
    HSCHK(noise_gpu_hs_set_key(ini.hs, NOISE_GPU_HS_S, sa.p, 0, nullptr));
    HSCHK(noise_gpu_hs_set_key(res.hs, NOISE_GPU_HS_S, sb.p, 0, nullptr));
    auto pre_has = [](const std::vector<PatternToken> &t, PatternToken x) {
      for (PatternToken y : t) if (y == x) return true;
      return false;
    };
    if (pre_has(prog.pre_r, PatternToken::S)) HSCHK(noise_gpu_hs_set_key(ini.hs, NOISE_GPU_HS_RS, pb.p, 0, nullptr));
    if (pre_has(prog.pre_i, PatternToken::S)) HSCHK(noise_gpu_hs_set_key(res.hs, NOISE_GPU_HS_RS, pa.p, 0, nullptr));
    if (prog.npsk) {
      HSCHK(noise_gpu_hs_set_psks(ini.hs, psk.p, nullptr));
      HSCHK(noise_gpu_hs_set_psks(res.hs, psk.p, nullptr));
    }
    HSCHK(noise_gpu_hs_start(ini.hs, nullptr, nullptr));
    HSCHK(noise_gpu_hs_start(res.hs, nullptr, nullptr));
    for (std::size_t m = 0; m < prog.msgs.size(); ++m) {
      const bool init_sends = prog.one_way || m % 2 == 0;
      noise_gpu_hs *w = init_sends ? ini.hs : res.hs, *rd = init_sends ? res.hs : ini.hs;
      noise_gpu_hs_info info;
      HSCHK(noise_gpu_hs_info_get(w, &info));
      noise_gpu_span ms{};
      ms.base = msg.p;
      ms.stride = cap;
      HSCHK(noise_gpu_hs_write_message(w, nullptr, &ms, nullptr, nullptr));
      ms.len_all = info.overhead;
      HSCHK(noise_gpu_hs_read_message(rd, &ms, nullptr, nullptr, nullptr, nullptr));
    }
    HSCHK(noise_gpu_hs_split(ini.hs, k1.p, k2.p, nullptr, nullptr, nullptr));
    HSCHK(noise_gpu_hs_split(res.hs, k1.p, k2.p, nullptr, nullptr, nullptr));
    HSCHK(noise_gpu_hs_status(res.hs, st.p, nullptr));
    HIPCHK(hipEventRecord(e1, nullptr));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<std::uint8_t> sv(n);
    st.get(sv.data(), n);
    for (std::uint8_t x : sv)
      if (x) throw std::runtime_error("a benchmark session failed");
    if (r > 0) best = std::min(best, (double)ms);
  }
  std::printf("{\"pattern\": \"%s\", \"sessions\": %zu, \"ms\": %.3f, \"handshakes_per_s\": %.0f}\n",
              pattern.c_str(), n, best, n / (best * 1e-3));
  return 0;
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
    } else if (cmd == "batch_vectors" && argc == 3) {
      return run_batch_vectors(argv[2]);
    } else if (cmd == "batch_check" && argc == 5) {
      return run_batch_check(argv[2], std::stoul(argv[3]), (unsigned)std::stoul(argv[4]));
    } else if (cmd == "batch_bench" && argc == 5) {
      return run_batch_bench(argv[2], std::stoul(argv[3]), std::atoi(argv[4]));
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
