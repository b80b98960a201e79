// crypto.cpp -- BLAKE2b, HMAC/HKDF and X25519 for the host-side Noise
// handshake (noise_amd/crypto.hpp).  Written from the specifications:
//   BLAKE2b   RFC 7693 §3.2-3.3 (G, compression F, 12 rounds, SIGMA)
//   HMAC      RFC 2104 with the hash's 128-byte block
//   HKDF      Noise rev34 §4.3 (HMAC-HASH, 2 or 3 outputs)
//   X25519    RFC 7748 §5 (clamped scalar, Montgomery ladder, a24 = 121665)
// Field arithmetic mod 2^255-19 in five 51-bit limbs with 128-bit products.
#include "noise_amd/crypto.hpp"

#include <sys/random.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace noise::crypto {

// ---- BLAKE2b ---------------------------------------------------------------
namespace {
constexpr std::uint64_t kIv[8] = {
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
    0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
    0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
constexpr std::uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

inline std::uint64_t rotr64(std::uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline std::uint64_t load64(const std::uint8_t *p) {
  std::uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
inline void store64(std::uint8_t *p, std::uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (std::uint8_t)(v >> (8 * i));
}
}  // namespace

Blake2b::Blake2b(std::size_t outlen) : outlen_(outlen) {
  if (outlen == 0 || outlen > kHashLen) throw std::invalid_argument("blake2b: output length");
  for (int i = 0; i < 8; ++i) h_[i] = kIv[i];
  h_[0] ^= 0x01010000ull ^ (std::uint64_t)outlen;  // depth 1, fanout 1, no key
}

void Blake2b::compress(bool last) {
  std::uint64_t v[16], m[16];
  for (int i = 0; i < 16; ++i) m[i] = load64(buf_ + 8 * i);
  for (int i = 0; i < 8; ++i) {
    v[i] = h_[i];
    v[i + 8] = kIv[i];
  }
  v[12] ^= t_[0];
  v[13] ^= t_[1];
  if (last) v[14] = ~v[14];
  auto G = [&](int a, int b, int c, int d, std::uint64_t x, std::uint64_t y) {
    v[a] = v[a] + v[b] + x;
    v[d] = rotr64(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];
    v[b] = rotr64(v[b] ^ v[c], 24);
    v[a] = v[a] + v[b] + y;
    v[d] = rotr64(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rotr64(v[b] ^ v[c], 63);
  };
  for (int r = 0; r < 12; ++r) {
    const std::uint8_t *s = kSigma[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) h_[i] ^= v[i] ^ v[i + 8];
  wipe(v, sizeof v);
  wipe(m, sizeof m);
}

void Blake2b::update(const std::uint8_t *p, std::size_t n) {
  while (n > 0) {
    if (fill_ == kBlockLen) {  // a full buffer is compressed only once more input arrives
      t_[0] += kBlockLen;
      if (t_[0] < kBlockLen) ++t_[1];
      compress(false);
      fill_ = 0;
    }
    const std::size_t take = n < kBlockLen - fill_ ? n : kBlockLen - fill_;
    std::memcpy(buf_ + fill_, p, take);
    fill_ += take;
    p += take;
    n -= take;
  }
}

void Blake2b::final(std::uint8_t *out) {
  t_[0] += fill_;
  if (t_[0] < fill_) ++t_[1];
  std::memset(buf_ + fill_, 0, kBlockLen - fill_);
  compress(true);
  std::uint8_t full[kHashLen];
  for (int i = 0; i < 8; ++i) store64(full + 8 * i, h_[i]);
  std::memcpy(out, full, outlen_);
  wipe(full, sizeof full);
  wipe(h_, sizeof h_);
  wipe(buf_, sizeof buf_);
}

Hash blake2b(const std::uint8_t *p, std::size_t n) {
  Blake2b b;
  b.update(p, n);
  Hash h;
  b.final(h.data());
  return h;
}

Hash hmac(const std::uint8_t *key, std::size_t key_len, const std::uint8_t *a,
          std::size_t a_len, const std::uint8_t *b, std::size_t b_len) {
  std::uint8_t k[kBlockLen] = {0};
  if (key_len > kBlockLen) {
    const Hash kh = blake2b(key, key_len);
    std::memcpy(k, kh.data(), kHashLen);
  } else if (key_len) {
    std::memcpy(k, key, key_len);
  }
  std::uint8_t pad[kBlockLen];
  for (std::size_t i = 0; i < kBlockLen; ++i) pad[i] = k[i] ^ 0x36;
  Blake2b inner;
  inner.update(pad, kBlockLen);
  if (a_len) inner.update(a, a_len);
  if (b_len) inner.update(b, b_len);
  Hash ih;
  inner.final(ih.data());
  for (std::size_t i = 0; i < kBlockLen; ++i) pad[i] = k[i] ^ 0x5c;
  Blake2b outer;
  outer.update(pad, kBlockLen);
  outer.update(ih.data(), kHashLen);
  Hash out;
  outer.final(out.data());
  wipe(k, sizeof k);
  wipe(pad, sizeof pad);
  wipe(ih.data(), ih.size());
  return out;
}

void hkdf(const Hash &ck, const std::uint8_t *ikm, std::size_t ikm_len, Hash *out1,
          Hash *out2, Hash *out3) {
  Hash temp = hmac(ck.data(), kHashLen, ikm, ikm_len);
  const std::uint8_t one = 1, two = 2, three = 3;
  const Hash o1 = hmac(temp.data(), kHashLen, &one, 1);
  const Hash o2 = hmac(temp.data(), kHashLen, o1.data(), kHashLen, &two, 1);
  if (out3) *out3 = hmac(temp.data(), kHashLen, o2.data(), kHashLen, &three, 1);
  *out1 = o1;
  *out2 = o2;
  wipe(temp.data(), temp.size());
}

// ---- X25519 ----------------------------------------------------------------
namespace {
using u128 = unsigned __int128;
using Fe = std::uint64_t[5];
constexpr std::uint64_t kM51 = (1ull << 51) - 1;

void fe_copy(Fe h, const Fe f) { std::memcpy(h, f, sizeof(Fe)); }

void fe_frombytes(Fe h, const std::uint8_t s[32]) {
  h[0] = load64(s) & kM51;
  h[1] = (load64(s + 6) >> 3) & kM51;
  h[2] = (load64(s + 12) >> 6) & kM51;
  h[3] = (load64(s + 19) >> 1) & kM51;
  h[4] = (load64(s + 24) >> 12) & kM51;  // the top bit is ignored (RFC 7748 §5)
}

void fe_carry(Fe h) {
  std::uint64_t c;
  c = h[0] >> 51; h[0] &= kM51; h[1] += c;
  c = h[1] >> 51; h[1] &= kM51; h[2] += c;
  c = h[2] >> 51; h[2] &= kM51; h[3] += c;
  c = h[3] >> 51; h[3] &= kM51; h[4] += c;
  c = h[4] >> 51; h[4] &= kM51; h[0] += 19 * c;
  c = h[0] >> 51; h[0] &= kM51; h[1] += c;
}

void fe_add(Fe h, const Fe f, const Fe g) {
  for (int i = 0; i < 5; ++i) h[i] = f[i] + g[i];
  fe_carry(h);
}

void fe_sub(Fe h, const Fe f, const Fe g) {  // f + 4p - g, limbs of g < 2^53
  h[0] = f[0] + 0x1FFFFFFFFFFFB4ull - g[0];
  for (int i = 1; i < 5; ++i) h[i] = f[i] + 0x1FFFFFFFFFFFFCull - g[i];
  fe_carry(h);
}

void fe_mul(Fe h, const Fe f, const Fe g) {
  const std::uint64_t g1 = 19 * g[1], g2 = 19 * g[2], g3 = 19 * g[3], g4 = 19 * g[4];
  u128 r0 = (u128)f[0] * g[0] + (u128)f[1] * g4 + (u128)f[2] * g3 + (u128)f[3] * g2 + (u128)f[4] * g1;
  u128 r1 = (u128)f[0] * g[1] + (u128)f[1] * g[0] + (u128)f[2] * g4 + (u128)f[3] * g3 + (u128)f[4] * g2;
  u128 r2 = (u128)f[0] * g[2] + (u128)f[1] * g[1] + (u128)f[2] * g[0] + (u128)f[3] * g4 + (u128)f[4] * g3;
  u128 r3 = (u128)f[0] * g[3] + (u128)f[1] * g[2] + (u128)f[2] * g[1] + (u128)f[3] * g[0] + (u128)f[4] * g4;
  u128 r4 = (u128)f[0] * g[4] + (u128)f[1] * g[3] + (u128)f[2] * g[2] + (u128)f[3] * g[1] + (u128)f[4] * g[0];
  r1 += (std::uint64_t)(r0 >> 51);
  r2 += (std::uint64_t)(r1 >> 51);
  r3 += (std::uint64_t)(r2 >> 51);
  r4 += (std::uint64_t)(r3 >> 51);
  h[0] = (std::uint64_t)r0 & kM51;
  h[1] = (std::uint64_t)r1 & kM51;
  h[2] = (std::uint64_t)r2 & kM51;
  h[3] = (std::uint64_t)r3 & kM51;
  h[4] = (std::uint64_t)r4 & kM51;
  h[0] += 19 * (std::uint64_t)(r4 >> 51);
  const std::uint64_t c = h[0] >> 51;
  h[0] &= kM51;
  h[1] += c;
}

void fe_sq(Fe h, const Fe f) { fe_mul(h, f, f); }

void fe_mul_small(Fe h, const Fe f, std::uint64_t k) {
  u128 c = 0;
  for (int i = 0; i < 5; ++i) {
    c += (u128)f[i] * k;
    h[i] = (std::uint64_t)c & kM51;
    c >>= 51;
  }
  h[0] += 19 * (std::uint64_t)c;
  fe_carry(h);
}

void fe_invert(Fe out, const Fe z) {  // z^(p-2), p-2 = 2^255 - 21
  Fe r;
  fe_copy(r, z);
  for (int i = 253; i >= 0; --i) {  // bit 254 is the leading one
    fe_sq(r, r);
    const bool bit = i >= 5 || ((0x0Bu >> i) & 1u);  // low 5 bits of p-2: 01011
    if (bit) fe_mul(r, r, z);
  }
  fe_copy(out, r);
}

void fe_tobytes(std::uint8_t s[32], const Fe f) {
  Fe h;
  fe_copy(h, f);
  fe_carry(h);
  fe_carry(h);
  // subtract p once if h >= p: q = 1 iff h + 19 >= 2^255
  std::uint64_t q = (h[0] + 19) >> 51;
  q = (h[1] + q) >> 51;
  q = (h[2] + q) >> 51;
  q = (h[3] + q) >> 51;
  q = (h[4] + q) >> 51;
  h[0] += 19 * q;
  std::uint64_t c = h[0] >> 51; h[0] &= kM51; h[1] += c;
  c = h[1] >> 51; h[1] &= kM51; h[2] += c;
  c = h[2] >> 51; h[2] &= kM51; h[3] += c;
  c = h[3] >> 51; h[3] &= kM51; h[4] += c;
  h[4] &= kM51;
  const std::uint64_t w0 = h[0] | (h[1] << 51), w1 = (h[1] >> 13) | (h[2] << 38),
                      w2 = (h[2] >> 26) | (h[3] << 25), w3 = (h[3] >> 39) | (h[4] << 12);
  store64(s, w0);
  store64(s + 8, w1);
  store64(s + 16, w2);
  store64(s + 24, w3);
}

void fe_cswap(Fe a, Fe b, std::uint64_t swap) {
  const std::uint64_t mask = 0 - swap;
  for (int i = 0; i < 5; ++i) {
    const std::uint64_t t = mask & (a[i] ^ b[i]);
    a[i] ^= t;
    b[i] ^= t;
  }
}
}  // namespace

Key32 x25519(const Key32 &scalar, const Key32 &u) {
  std::uint8_t k[32];
  std::memcpy(k, scalar.data(), 32);
  k[0] &= 248;
  k[31] &= 127;
  k[31] |= 64;
  Fe x1, x2 = {1, 0, 0, 0, 0}, z2 = {0, 0, 0, 0, 0}, x3, z3 = {1, 0, 0, 0, 0};
  fe_frombytes(x1, u.data());
  fe_copy(x3, x1);
  std::uint64_t swap = 0;
  Fe a, aa, b, bb, e, c, d, da, cb, t;
  for (int pos = 254; pos >= 0; --pos) {
    const std::uint64_t bit = (k[pos >> 3] >> (pos & 7)) & 1u;
    swap ^= bit;
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    swap = bit;
    fe_add(a, x2, z2);
    fe_sq(aa, a);
    fe_sub(b, x2, z2);
    fe_sq(bb, b);
    fe_sub(e, aa, bb);
    fe_add(c, x3, z3);
    fe_sub(d, x3, z3);
    fe_mul(da, d, a);
    fe_mul(cb, c, b);
    fe_add(t, da, cb);
    fe_sq(x3, t);
    fe_sub(t, da, cb);
    fe_sq(t, t);
    fe_mul(z3, x1, t);
    fe_mul(x2, aa, bb);
    fe_mul_small(t, e, 121665);
    fe_add(t, aa, t);
    fe_mul(z2, e, t);
  }
  fe_cswap(x2, x3, swap);
  fe_cswap(z2, z3, swap);
  fe_invert(z2, z2);
  fe_mul(x2, x2, z2);
  Key32 out;
  fe_tobytes(out.data(), x2);
  wipe(k, sizeof k);
  return out;
}

Key32 x25519_base(const Key32 &scalar) {
  Key32 nine{};
  nine[0] = 9;
  return x25519(scalar, nine);
}

void random_bytes(std::uint8_t *p, std::size_t n) {
  while (n > 0) {
    const ssize_t r = getrandom(p, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("getrandom failed");
    }
    p += r;
    n -= (std::size_t)r;
  }
}

bool verify(const std::uint8_t *a, const std::uint8_t *b, std::size_t n) {
  std::uint8_t d = 0;
  for (std::size_t i = 0; i < n; ++i) d |= a[i] ^ b[i];
  return d == 0;
}

void wipe(void *p, std::size_t n) {
  volatile std::uint8_t *v = static_cast<volatile std::uint8_t *>(p);
  for (std::size_t i = 0; i < n; ++i) v[i] = 0;
}

}  // namespace noise::crypto
