// tests/cpp/ref_signatures.cpp -- a caller of the reference's free AEAD
// functions that knows only their declarations as the reference's library
// defines them (noise.cpp:202-204 and 254-256, namespace noise at
// noise.cpp:32): nothing from this build's headers.  Linked against
// libnoise_amd.so it must resolve both names, so the engine can replace
// noise.cpp:179-281 outright.
//   ref_signatures            -> calls both once; without a GPU the engine
//                                throws std::runtime_error, which is reported
#include <array>
#include <cstdint>
#include <cstdio>
#include <optional>
#include <stdexcept>
#include <vector>

namespace noise {
void encrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out);
void decrypt(std::array<std::uint8_t, 32> &k, std::uint64_t n,
             std::optional<std::vector<std::uint8_t>> ad,
             std::vector<std::uint8_t> &in_out);
}  // namespace noise

int main() {
  std::array<std::uint8_t, 32> k{};
  for (int i = 0; i < 32; ++i) k[i] = (std::uint8_t)i;
  std::vector<std::uint8_t> m = {1, 2, 3};
  try {
    noise::encrypt(k, 0, std::nullopt, m);
    std::array<std::uint8_t, 32> k2{};
    for (int i = 0; i < 32; ++i) k2[i] = (std::uint8_t)i;
    noise::decrypt(k2, 0, std::nullopt, m);
    std::printf("round trip %s\n", m == std::vector<std::uint8_t>({1, 2, 3}) ? "ok" : "FAILED");
    return m == std::vector<std::uint8_t>({1, 2, 3}) ? 0 : 1;
  } catch (const std::runtime_error &e) {
    std::printf("runtime_error: %s\n", e.what());
    return 3;
  }
}
