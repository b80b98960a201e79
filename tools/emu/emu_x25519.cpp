// emu_x25519.cpp -- the device X25519 code (csrc/x25519_device.hpp),
// unmodified, compiled as host C++ under ASan: the fixed-base public-key path
// (base_scalarmult: edwards25519 radix-16 table) against the Montgomery
// ladder with u = 9 and the host X25519 (host/crypto.cpp), on RFC 7748 §6.1
// and random scalars.  Test infrastructure (tests/test_emu_kernels.py).
//   emu_x25519 <count> <seed>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "hip/hip_runtime.h"
#include "noise_amd/crypto.hpp"
#include "x25519_device.hpp"

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200;
  std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 1);
  int fails = 0;
  for (int c = 0; c < n + 1; ++c) {
    std::array<std::uint8_t, 32> sk;
    if (c == 0) {  // RFC 7748 §6.1 Alice
      const char *hx = "77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a";
      for (int b = 0; b < 32; ++b) sk[b] = (std::uint8_t)std::stoul(std::string(hx + 2 * b, 2), nullptr, 16);
    } else {
      for (auto &b : sk) b = (std::uint8_t)rng();
      if (c % 7 == 1) sk.fill((std::uint8_t)(c % 3 == 0 ? 0xff : 0x00));  // extremes
    }
    std::uint32_t k[8], u9[8] = {9, 0, 0, 0, 0, 0, 0, 0}, a[8], l[8];
    std::memcpy(k, sk.data(), 32);
    noise_amd::x25519::base_scalarmult(a, k);
    noise_amd::x25519::scalarmult(l, k, u9);
    const auto h = noise::crypto::x25519_base(sk);
    const bool ok = std::memcmp(a, l, 32) == 0 && std::memcmp(a, h.data(), 32) == 0;
    if (c == 0) {
      const char *want = "8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a";
      char got[65];
      for (int b = 0; b < 32; ++b) std::snprintf(got + 2 * b, 3, "%02x", ((std::uint8_t *)a)[b]);
      if (std::strcmp(got, want) != 0) {
        std::printf("FAIL RFC 7748 6.1: %s\n", got);
        ++fails;
      }
    }
    if (!ok && fails++ < 10) std::printf("FAIL scalar %d\n", c);
  }
  std::printf("fixed-base public keys: %d scalars, %d failures: %s\n", n + 1, fails, fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
