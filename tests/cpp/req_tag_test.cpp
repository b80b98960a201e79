// tests/cpp/req_tag_test.cpp -- the resident request line's per-chunk check
// (noise-cpp_amd/csrc/launchers.hpp req_chunk_tag): a chunk
// whose 16-byte BAR store lands in part -- the new first word (seq ^ tag of
// the new payload) over stale payload words -- must not decode to the new
// seq.  Torn chunk 0 over small lengths / AD lengths / directions and nonces
// (structured values, the case XOR-of-rotations got wrong), stale payloads of
// zero (after the kernel's wipe) and of the previous request; the key chunks
// torn the same way.  Host-only: the tag is constexpr __host__ __device__.
//   g++ -std=c++20 -I tools/emu/include -I include -I noise-cpp_amd/csrc
#include <cstdint>
#include <cstdio>
#include <vector>

#include "launchers.hpp"

int main() {
  using noise_amd::req_chunk_tag;
  std::vector<uint32_t> metas, nonces;
  for (uint32_t len : {0u, 1u, 16u, 64u, 100u, 1024u, 1488u, 4032u})
    for (uint32_t ad : {0u, 32u, 64u})
      for (uint32_t dec : {0u, 1u}) metas.push_back(len | ad << 16 | dec << 30);
  for (uint32_t b = 0; b < 32; ++b) nonces.push_back(1u << b);
  for (uint32_t v = 0; v < 300; ++v) nonces.push_back(v);
  long pairs = 0, bad = 0;
  // chunk 0 {seq ^ tag(meta, nlo, nhi), meta, nlo, nhi}: torn over a zero
  // payload and over the previous request's payload (nonce - 1)
  for (uint32_t m : metas)
    for (uint32_t lo : nonces)
      for (uint32_t hi : {0u, 1u, 0x80000000u}) {
        const uint32_t t = req_chunk_tag(0u, m, lo, hi);
        ++pairs;
        if ((m | lo | hi) != 0u && t == req_chunk_tag(0u, 0u, 0u, 0u)) {  // (a payload of zeros is no tear)
          if (bad++ < 5) std::printf("torn over zeros: meta %08x nonce %08x:%08x\n", m, hi, lo);
        }
        if (lo != 0u) {
          ++pairs;
          if (t == req_chunk_tag(0u, m, lo - 1u, hi)) {
            if (bad++ < 5) std::printf("torn over the previous nonce: meta %08x nonce %08x:%08x\n", m, hi, lo);
          }
        }
      }
  // key chunks 1..3 {seq ^ tag(k0, k1, k2), ...}: single-word keys over zeros
  for (uint32_t c = 1; c <= 3; ++c)
    for (uint32_t b = 0; b < 32; ++b)
      for (int w = 0; w < 3; ++w) {
        const uint32_t k[3] = {w == 0 ? 1u << b : 0u, w == 1 ? 1u << b : 0u, w == 2 ? 1u << b : 0u};
        ++pairs;
        if (req_chunk_tag(c, k[0], k[1], k[2]) == req_chunk_tag(c, 0u, 0u, 0u)) ++bad;
      }
  // the linear tag's collision: len 64 with nonce 2^26
  const bool advice_case = req_chunk_tag(0u, 64u, 1u << 26, 0u) != req_chunk_tag(0u, 0u, 0u, 0u);
  std::printf("%ld torn chunks checked, %ld decode to the new seq; advice case %s\n", pairs, bad,
              advice_case ? "distinct" : "COLLIDES");
  return bad == 0 && advice_case ? 0 : 1;
}
