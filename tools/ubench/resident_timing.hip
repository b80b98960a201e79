// resident_timing.hip -- where a resident-mode single record (k_aead_resident,
// single_kernels.hip) spends its time, back to back like CipherState's
// consecutive encrypt_with_ad calls (so the speculation slot hits).  The
// product source built with NOISE_ONE_TIMING: s_memrealtime (100 MHz) stamps
// in the host image's done line at request detection, data landed, tag
// computed, stores issued, done word, and the end of the speculation that
// follows.  Host wall time per call as CipherState would see it (stage the
// record, ring, spin on the done word, copy the output out).
//   resident_timing [fine|host] -> one line per record size
#define NOISE_ONE_TIMING 1
#include "single_kernels.hip"

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

using namespace noise_amd;

int main(int argc, char **argv) {
  const bool hostreq = argc > 1 && !std::strcmp(argv[1], "host");
  uint8_t *h = nullptr, *d = nullptr, *hq = nullptr, *dq = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), kOneReqBytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0) != hipSuccess) return 1;
  std::memset(h, 0, kOneReqBytes);
  if (hostreq) {
    if (hipHostMalloc(reinterpret_cast<void **>(&hq), kOneReqBytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&dq), hq, 0) != hipSuccess) return 1;
    std::memset(hq, 0, kOneReqBytes);
  } else {
    if (hipExtMallocWithFlags(reinterpret_cast<void **>(&dq), kOneReqBytes, hipDeviceMallocFinegrained) != hipSuccess) return 1;
    hq = dq;
    if (hipMemset(dq, 0, kOneReqBytes) != hipSuccess) return 1;
  }
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  reinterpret_cast<uint32_t *>(h)[2] = 1u;  // alive
  if (launch_aead_resident(dq, d, 0u, 2000000u, st) != hipSuccess) return 2;
  uint32_t key[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  uint32_t seq = 0;
  uint64_t nonce = 1000;
  std::printf("# %s request image; us: detect->data  data->tag  tag->stores  stores->done | spec "
              "| prev done -> detect | host wall per call\n", hostreq ? "host" : "fine-grained");
  std::vector<uint8_t> out(70000);
  for (uint32_t L : {64u, 1024u, 1472u, 3000u, 16384u}) {
    const OneLayout lay = one_layout(0, L);
    std::vector<double> ph[4], spec, idle, wall, unp, hitv;
    uint64_t prev_spec_end = 0;
    for (int it = 0; it < 200; ++it) {
      std::vector<uint8_t> pt(L);
      for (uint32_t i = 0; i < L; ++i) pt[i] = (uint8_t)(i * 7 + it);
      const auto t0 = std::chrono::steady_clock::now();
      const uint32_t n_inl = req_inline_chunks(0, L, false);
      if (n_inl) {
        std::vector<uint8_t> im(12 * n_inl + 16, 0);
        std::memcpy(im.data(), pt.data(), L);
        for (uint32_t k = 0; k < n_inl; ++k) {
          uint32_t w[3];
          std::memcpy(w, im.data() + 12 * k, 12);
          _mm_store_si128(reinterpret_cast<__m128i *>(hq) + 4 + k,
                          _mm_setr_epi32((int)(seq + 1), (int)w[0], (int)w[1], (int)w[2]));
        }
      } else {
        std::memcpy(hq + kReqStageOff + lay.in, pt.data(), L);
      }
      _mm_sfence();
      const uint32_t s = ++seq;
      __m128i *q = reinterpret_cast<__m128i *>(hq);
      _mm_store_si128(q + 1, _mm_setr_epi32((int)s, (int)key[0], (int)key[1], (int)key[2]));
      _mm_store_si128(q + 2, _mm_setr_epi32((int)s, (int)key[3], (int)key[4], (int)key[5]));
      _mm_store_si128(q + 3, _mm_setr_epi32((int)s, (int)key[6], (int)key[7], 0));
      _mm_store_si128(q + 0, _mm_setr_epi32((int)s, (int)L, (int)(uint32_t)nonce, (int)(uint32_t)(nonce >> 32)));
      _mm_sfence();
      ++nonce;
      volatile uint32_t *done = reinterpret_cast<volatile uint32_t *>(h);
      uint64_t spins = 0;
      while (*done != s && ++spins < 2000000000ull) {
      }
      if (*done != s) { std::printf("no answer\n"); return 3; }
      std::memcpy(out.data(), h + lay.out, L + 16);
      const auto t1 = std::chrono::steady_clock::now();
      // the stamps now in the done line are the PREVIOUS request's (the
      // kernel copies them out after its speculation, off the critical path):
      // [0] detect [1] data in LDS [3] tag [4] stores issued [5] done [6] spec end
      const volatile uint64_t *ts = reinterpret_cast<const volatile uint64_t *>(h + kOneTsOff);
      const uint64_t t_det = ts[0], t_data = ts[1], t_tag = ts[3], t_st = ts[4], t_done = ts[5],
                     t_spec = ts[6], t_unp = ts[2], t_hit = ts[7];
      if (it >= 10) { unp.push_back((t_unp - t_det) * 0.01); hitv.push_back((t_hit - t_det) * 0.01); }
      if (it >= 10) {
        ph[0].push_back((t_data - t_det) * 0.01);
        ph[1].push_back((t_tag - t_data) * 0.01);
        ph[2].push_back((t_st - t_tag) * 0.01);
        ph[3].push_back((t_done - t_st) * 0.01);
        spec.push_back((t_spec - t_done) * 0.01);
        if (prev_spec_end) idle.push_back(((double)(int64_t)(t_det - prev_spec_end)) * 0.01);
        wall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      prev_spec_end = t_done;  // this (previous) request's done -> the next one's detect
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return -1.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    std::printf("L %5u: %.2f %.2f %.2f %.2f | %.2f | %.2f | %.2f   (detect->unpacked %.2f, ->slot chosen %.2f)\n", L, med(ph[0]), med(ph[1]),
                med(ph[2]), med(ph[3]), med(spec), med(idle), med(wall), med(unp), med(hitv));
  }
  reinterpret_cast<OneRing *>(h + kOneRingOff)->stop = 1u;
  (void)hipStreamSynchronize(st);
  return 0;
}
