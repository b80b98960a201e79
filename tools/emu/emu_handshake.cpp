// emu_handshake.cpp -- the batched-handshake kernels (csrc/handshake_kernels.hip)
// and their host driver (csrc/handshake_batch.hip), unmodified, compiled as
// host C++ against the emulation header and run under AddressSanitizer:
// the reference's vectors (tests/golden/handshake_vectors.tsv) replayed
// through noise_gpu_hs_* with "device" buffers in host memory -- every
// handshake message, the handshake hashes, both sides' split keys, and the
// transport records under those keys against the CPU oracle.  Test
// infrastructure (tests/test_emu_kernels.py); the product never runs here.
//   emu_handshake <vectors.tsv> [max_vectors]
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "hip/hip_runtime.h"
#include "noise_amd/handshake.hpp"
#include "noise_gpu.h"

extern "C" void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                                     size_t ad_len, const uint8_t *pt, size_t len, uint8_t *out);

// the C-ABI helpers handshake_batch.hip links against (noise_gpu_api.hip on the GPU)
static std::string g_err;
namespace noise_amd {
int api_hip_fail(hipError_t, const char *what) {
  g_err = what;
  return NOISE_GPU_E_HIP;
}
int api_arg_fail(const char *msg) {
  g_err = msg;
  return NOISE_GPU_E_ARG;
}
int api_check_device() { return NOISE_GPU_OK; }
}  // namespace noise_amd

using bytes = std::vector<std::uint8_t>;

static bytes unhex(const std::string &s) {
  if (s == "-") return {};
  bytes b(s.size() / 2);
  for (std::size_t i = 0; i < b.size(); ++i) b[i] = (std::uint8_t)std::stoul(s.substr(2 * i, 2), nullptr, 16);
  return b;
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
  std::string name, pattern, f[11];
  std::vector<std::pair<bytes, bytes>> msgs;
};

#define CHK(x)                                                              \
  do {                                                                      \
    if ((x) != 0) throw std::runtime_error(std::string(#x) + ": " + g_err); \
  } while (0)

// ragged per-session buffer at 16-aligned offsets ("device" = host here)
struct Ragged {
  std::vector<std::uint64_t> off;
  std::vector<std::uint32_t> len;
  bytes data;
  Ragged(const std::vector<bytes> &items, std::size_t room) {
    std::uint64_t o = 0;
    for (const bytes &b : items) {
      off.push_back(o);
      len.push_back((std::uint32_t)b.size());
      o += (b.size() + room + 15) & ~std::size_t(15);
    }
    data.assign(o + 16, 0);
    for (std::size_t i = 0; i < items.size(); ++i)
      if (!items[i].empty()) std::memcpy(data.data() + off[i], items[i].data(), items[i].size());
  }
  noise_gpu_span span() {
    noise_gpu_span s{};
    s.base = data.data();
    s.off = off.data();
    s.len = len.data();
    return s;
  }
};

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::size_t maxv = argc > 2 ? std::stoul(argv[2]) : 1000;
  std::ifstream in(argv[1]);
  std::vector<Vec> all;
  std::string line;
  while (std::getline(in, line) && all.size() < maxv) {
    if (line.empty()) continue;
    const auto cols = split(line, '\t');
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
  int fails = 0, hashes = 0, transport = 0, messages = 0;
  for (const Vec &v : all) {
    try {
      const auto prog = noise::detail::parse_pattern(v.pattern);
      noise_gpu_hs *side[2] = {nullptr, nullptr};
      for (int r = 0; r < 2; ++r) {
        const int o = r ? 5 : 0;
        CHK(noise_gpu_hs_create(v.pattern.c_str(), r == 0, 1, &side[r]));
        const int slot_of[3] = {NOISE_GPU_HS_S, NOISE_GPU_HS_E, NOISE_GPU_HS_RS};
        for (int k = 0; k < 3; ++k) {
          bytes key = unhex(v.f[o + 2 + k]);
          if (!key.empty()) CHK(noise_gpu_hs_set_key(side[r], slot_of[k], key.data(), 32, nullptr));
        }
        bytes psks;
        if (v.f[o + 1] != "-")
          for (const std::string &p : split(v.f[o + 1], ',')) {
            const bytes b = unhex(p);
            psks.insert(psks.end(), b.begin(), b.end());
          }
        if (!psks.empty()) CHK(noise_gpu_hs_set_psks(side[r], psks.data(), nullptr));
        Ragged pro({unhex(v.f[o])}, 0);
        noise_gpu_span ps = pro.span();
        CHK(noise_gpu_hs_start(side[r], &ps, nullptr));
      }
      const std::size_t nhs = prog.msgs.size();
      for (std::size_t m = 0; m < nhs; ++m) {
        const bool init_sends = prog.one_way || m % 2 == 0;
        noise_gpu_hs *w = side[init_sends ? 0 : 1], *rd = side[init_sends ? 1 : 0];
        noise_gpu_hs_info info;
        CHK(noise_gpu_hs_info_get(w, &info));
        Ragged pay({v.msgs[m].first}, 0), msg({v.msgs[m].first}, info.overhead), out({v.msgs[m].first}, 16);
        std::uint32_t mlen = 0, plen = 0;
        std::uint8_t st = 9;
        noise_gpu_span ps = pay.span(), ms = msg.span(), os = out.span();
        CHK(noise_gpu_hs_write_message(w, &ps, &ms, &mlen, nullptr));
        const bytes wire(msg.data.begin(), msg.data.begin() + mlen);
        if (wire != v.msgs[m].second) throw std::runtime_error("message " + std::to_string(m) + " differs");
        msg.len[0] = mlen;
        ms = msg.span();
        CHK(noise_gpu_hs_read_message(rd, &ms, &os, &plen, &st, nullptr));
        if (st != 0 || bytes(out.data.begin(), out.data.begin() + plen) != v.msgs[m].first)
          throw std::runtime_error("payload " + std::to_string(m) + " not recovered");
        ++messages;
      }
      alignas(16) std::uint8_t k[2][2][32], h[2][64];
      for (int r = 0; r < 2; ++r) CHK(noise_gpu_hs_split(side[r], k[r][0], k[r][1], h[r], nullptr, nullptr));
      if (std::memcmp(k[0], k[1], 64) != 0 || std::memcmp(h[0], h[1], 64) != 0)
        throw std::runtime_error("the sides' split differs");
      if (v.f[10] != "-") {
        if (bytes(h[0], h[0] + 64) != unhex(v.f[10])) throw std::runtime_error("handshake hash differs");
        ++hashes;
      }
      std::uint64_t n[2] = {0, 0};
      bytes ct(65535 + 16);
      for (std::size_t m = nhs; m < v.msgs.size(); ++m) {
        const int dir = (prog.one_way || m % 2 == 0) ? 0 : 1;  // k1: initiator -> responder
        const bytes &pt = v.msgs[m].first;
        oracle_noise_encrypt(k[0][dir], n[dir]++, nullptr, 0, pt.data(), pt.size(), ct.data());
        if (bytes(ct.begin(), ct.begin() + pt.size() + 16) != v.msgs[m].second)
          throw std::runtime_error("transport message differs");
        ++transport;
      }
      for (auto *s : side) noise_gpu_hs_destroy(s);
    } catch (const std::exception &e) {
      if (fails++ < 20) std::printf("FAIL %s: %s\n", v.name.c_str(), e.what());
    }
  }
  std::printf("emulated batched handshakes: vectors %zu, failed %d, messages %d, handshake hashes %d, "
              "transport records %d: %s\n", all.size(), fails, messages, hashes, transport,
              fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
