// config1_bench -- BASELINE config 1 through the build's drop-in classes:
// the XX loopback handshake of examples/Noise_XX_25519_ChaChaPoly_Blake2b.cpp
// (26-57: both parties in one process, fresh static keys) and then
// `records` transport records of `len` bytes each way, sent the way the
// reference's users send them (examples/...:58-75): one
// CipherState::encrypt_with_ad / decrypt_with_ad call per record.  Every
// AEAD runs on the GPU (noise-cpp_amd/lib/libnoise_amd.so); bench.py times
// the reference's Monocypher beside it (oracle/_ref) in the same run.
//
//   config1_bench <records> <len> [resident]   -> one JSON line on stdout
//
// "resident": the single-record calls go through the resident latency
// workgroup (noise_gpu_set_resident) instead of one kernel launch each; it is
// switched off again at the end (the shutdown path), reported as "stopped".
//
// Also reported: the same records through encrypt_batch / decrypt_batch
// (one GPU call per direction), and the per-call latency of
// encrypt_with_ad / decrypt_with_ad at several record sizes.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "noise_amd/handshake.hpp"
#include "noise_gpu.h"

using bytes = std::vector<std::uint8_t>;
using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

struct Pair {
  noise::CipherState i_send, i_recv, r_send, r_recv;
};

static double handshake(Pair &p) {
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
  std::tie(p.i_send, p.i_recv) = ini.finalize();
  std::tie(p.r_recv, p.r_send) = res.finalize();
  return secs(t0, clk::now());
}

static std::vector<bytes> make_records(int records, int len) {
  std::vector<bytes> v(records, bytes(len));
  for (int i = 0; i < records; ++i)
    for (int j = 0; j < len; ++j) v[i][j] = (std::uint8_t)(7 * j + 3 + i);
  return v;
}

// records through per-record calls; returns {enc seconds, dec seconds}
static std::pair<double, double> per_record(noise::CipherState &snd, noise::CipherState &rcv,
                                            std::vector<bytes> &recs, const std::vector<bytes> &orig) {
  const auto t0 = clk::now();
  for (auto &m : recs) snd.encrypt_with_ad(m);
  const auto t1 = clk::now();
  for (auto &m : recs) rcv.decrypt_with_ad(m);
  const auto t2 = clk::now();
  if (recs != orig) throw std::runtime_error("per-record round trip differs");
  return {secs(t0, t1), secs(t1, t2)};
}

int main(int argc, char **argv) {
  const int records = argc > 1 ? std::atoi(argv[1]) : 1000;
  const int len = argc > 2 ? std::atoi(argv[2]) : 1024;
  const bool resident = argc > 3 && std::string(argv[3]) == "resident";
  try {
    if (resident && noise_gpu_set_resident(1, 0) != NOISE_GPU_OK)
      throw std::runtime_error(std::string("set_resident: ") + noise_gpu_last_error());
    Pair warm;
    handshake(warm);  // device init, staging, code objects
    {
      auto w = make_records(16, len);
      const auto o = w;
      per_record(warm.i_send, warm.r_recv, w, o);
      auto wb = make_records(records, len);  // the batch path's staging, once
      warm.i_send.encrypt_batch(wb);
      warm.r_recv.decrypt_batch(wb);
    }
    // handshake: best of 5 (each one a fresh pair of parties)
    double hs = 1e9;
    Pair p;
    for (int i = 0; i < 5; ++i) {
      Pair q;
      hs = std::min(hs, handshake(q));
      if (i == 4) p = q;
    }
    const std::vector<bytes> orig = make_records(records, len);
    auto recs = orig;
    const auto [e1, d1] = per_record(p.i_send, p.r_recv, recs, orig);  // initiator -> responder
    const auto [e2, d2] = per_record(p.r_send, p.i_recv, recs, orig);  // responder -> initiator
    // the same records through one batch call per direction
    const auto b0 = clk::now();
    p.i_send.encrypt_batch(recs);
    const auto b1 = clk::now();
    p.r_recv.decrypt_batch(recs);
    const auto b2 = clk::now();
    if (recs != orig) throw std::runtime_error("batch round trip differs");
    // per-call latency by record size (median of 50 calls each way)
    std::string lat = "{";
    const int sizes[] = {64, 1024, 4096, 16384, 65519};
    for (int si = 0; si < 5; ++si) {
      const int L = sizes[si];
      std::vector<double> te, td;
      bytes m(L, 0x5a);
      for (int i = 0; i < 51; ++i) {
        const auto a = clk::now();
        p.i_send.encrypt_with_ad(m);
        const auto b = clk::now();
        p.r_recv.decrypt_with_ad(m);
        const auto c = clk::now();
        te.push_back(secs(a, b));
        td.push_back(secs(b, c));
      }
      std::sort(te.begin(), te.end());
      std::sort(td.begin(), td.end());
      char buf[160];
      std::snprintf(buf, sizeof buf, "%s\"%d\": {\"encrypt_us\": %.2f, \"decrypt_us\": %.2f}",
                    si ? ", " : "", L, te[25] * 1e6, td[25] * 1e6);
      lat += buf;
    }
    lat += "}";
    bool stopped = true;
    if (resident) {  // shutdown path: the workgroup leaves, later calls launch again
      stopped = noise_gpu_set_resident(0, 0) == NOISE_GPU_OK;
      bytes m(len, 1);
      const bytes o = m;
      p.i_send.encrypt_with_ad(m);
      p.r_recv.decrypt_with_ad(m);
      stopped = stopped && m == o;
    }
    std::printf("{\"mode\": \"%s\", \"stopped\": %s, \"handshake_ms\": %.4f, \"records\": %d, \"record_bytes\": %d, "
                "\"per_record\": {\"encrypt_ms\": %.3f, \"decrypt_ms\": %.3f, "
                "\"encrypt_ms_back\": %.3f, \"decrypt_ms_back\": %.3f, \"per_record_us\": %.3f}, "
                "\"batch\": {\"encrypt_ms\": %.3f, \"decrypt_ms\": %.3f}, "
                "\"latency_by_size\": %s, \"ok\": true}\n",
                resident ? "resident" : "launch", stopped ? "true" : "false", hs * 1e3, records, len, e1 * 1e3, d1 * 1e3, e2 * 1e3, d2 * 1e3,
                (e1 + d1 + e2 + d2) / 4 / records * 1e6, secs(b0, b1) * 1e3, secs(b1, b2) * 1e3,
                lat.c_str());
  } catch (const std::exception &e) {
    std::fprintf(stderr, "config1_bench: %s\n", e.what());
    return 1;
  }
  return 0;
}
