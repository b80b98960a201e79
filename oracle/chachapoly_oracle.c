/*
 * oracle/chachapoly_oracle.c -- CPU restatement of the reference's
 * Noise transport-record AEAD.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this (as liboracle.so).  The product (noise-cpp_amd/, include/) never
 * links or calls it; the GPU path fails loudly rather than fall back here.
 *
 * What it restates (reference = ethindp/noise-cpp @ 2025-09-05):
 *   oracle_noise_encrypt   noise::encrypt            noise.cpp:202-224
 *                          crypto_aead_init_ietf     monocypher.c:2891-2897
 *                          crypto_aead_write         monocypher.c:2899-2910
 *   oracle_noise_decrypt   noise::decrypt            noise.cpp:254-281
 *                          crypto_aead_read          monocypher.c:2912-2929
 *   oracle_chacha20_block  chacha20_rounds + feed-forward in
 *                          crypto_chacha20_djb       monocypher.c:178-200, 219-276
 *   poly1305_*             crypto_poly1305_init/update/final, lock_auth
 *                                                    monocypher.c:366-440, 2858-2873
 *   oracle_rekey           CipherState::rekey        noise.cpp:429-439
 *   oracle_check_records / oracle_check_uniform: the above per record over
 *                          a whole GPU batch (full-size parity tests)
 *
 * The arithmetic is written independently (RFC 8439 structure; Poly1305 in
 * 3 x 44-bit limbs with 128-bit products, unlike monocypher's 5 x 32-bit
 * limbs), so agreement with oracle/_ref (monocypher itself) is a real
 * cross-check.  Parity pinning: tests/test_oracle.py checks this file
 * against all 1688 transport records and 1828 with-AD handshake records
 * derived from the reference's tests/vectors (tests/golden/), against the
 * SURVEY.md section 8(c) known-answer tests, and against monocypher.c
 * compiled from /root/reference (oracle/_ref) where that is present.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;

static uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
         (uint32_t)p[3] << 24;
}
static uint64_t ld64(const uint8_t *p) {
  return (uint64_t)ld32(p) | (uint64_t)ld32(p + 4) << 32;
}
static void st32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void st64(uint8_t *p, uint64_t v) {
  st32(p, (uint32_t)v); st32(p + 4, (uint32_t)(v >> 32));
}
static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* ChaCha20 block, IETF layout: words 12 = block counter, 13..15 = nonce.
 * Noise's nonce is 0^32 || LE64(n) (noise.cpp:207-215), so word 13 = 0,
 * 14 = lo32(n), 15 = hi32(n); monocypher's djb counter split
 * (monocypher.c:2895-2896, 224-227) gives the same words. */
void oracle_chacha20_block(const uint8_t key[32], uint32_t counter,
                           const uint8_t nonce12[12], uint8_t out[64]) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
  for (int i = 0; i < 8; ++i) s[4 + i] = ld32(key + 4 * i);
  s[12] = counter;
  for (int i = 0; i < 3; ++i) s[13 + i] = ld32(nonce12 + 4 * i);
  memcpy(x, s, sizeof x);
#define QR(a, b, c, d)                                              \
  x[a] += x[b]; x[d] = rol(x[d] ^ x[a], 16);                        \
  x[c] += x[d]; x[b] = rol(x[b] ^ x[c], 12);                        \
  x[a] += x[b]; x[d] = rol(x[d] ^ x[a], 8);                         \
  x[c] += x[d]; x[b] = rol(x[b] ^ x[c], 7);
  for (int r = 0; r < 10; ++r) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
#undef QR
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + s[i]);
}

/* ---- Poly1305: h = sum m_i r^(k-i+1) mod 2^130-5, tag = (h + s) mod 2^128.
 * Limbs of 44/44/42 bits. */
typedef struct {
  uint64_t r0, r1, r2, s1, s2; /* s_i = 20 * r_i (2^132 = 4 * 2^130 == 20) */
  uint64_t h0, h1, h2;
  uint64_t pad0, pad1;
} poly_t;

static void poly_init(poly_t *p, const uint8_t key[32]) {
  /* clamp r (monocypher.c:373-374) */
  uint64_t t0 = ld64(key) & 0x0ffffffc0fffffffull;
  uint64_t t1 = ld64(key + 8) & 0x0ffffffc0ffffffcull;
  p->r0 = t0 & 0xfffffffffffull;
  p->r1 = ((t0 >> 44) | (t1 << 20)) & 0xfffffffffffull;
  p->r2 = (t1 >> 24) & 0x3ffffffffffull;
  p->s1 = p->r1 * 20;
  p->s2 = p->r2 * 20;
  p->h0 = p->h1 = p->h2 = 0;
  p->pad0 = ld64(key + 16);
  p->pad1 = ld64(key + 24);
}

/* one full 16-byte block with the 2^128 bit set */
static void poly_block(poly_t *p, const uint8_t m[16]) {
  const uint64_t M44 = 0xfffffffffffull, M42 = 0x3ffffffffffull;
  uint64_t t0 = ld64(m), t1 = ld64(m + 8);
  uint64_t h0 = p->h0 + (t0 & M44);
  uint64_t h1 = p->h1 + (((t0 >> 44) | (t1 << 20)) & M44);
  uint64_t h2 = p->h2 + (((t1 >> 24) & M42) | (1ull << 40));
  u128 d0 = (u128)h0 * p->r0 + (u128)h1 * p->s2 + (u128)h2 * p->s1;
  u128 d1 = (u128)h0 * p->r1 + (u128)h1 * p->r0 + (u128)h2 * p->s2;
  u128 d2 = (u128)h0 * p->r2 + (u128)h1 * p->r1 + (u128)h2 * p->r0;
  uint64_t c;
  c = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & M44;
  d1 += c; c = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & M44;
  d2 += c; c = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & M42;
  h0 += c * 5; c = h0 >> 44; h0 &= M44;
  h1 += c;
  p->h0 = h0; p->h1 = h1; p->h2 = h2;
}

/* absorb `len` bytes zero-padded to a multiple of 16 (lock_auth's
 * update(x) + update(zero, gap(x,16)), monocypher.c:2866-2869) */
static void poly_padded(poly_t *p, const uint8_t *m, size_t len) {
  while (len >= 16) { poly_block(p, m); m += 16; len -= 16; }
  if (len) {
    uint8_t b[16] = {0};
    memcpy(b, m, len);
    poly_block(p, b);
  }
}

static void poly_final(poly_t *p, uint8_t tag[16]) {
  const uint64_t M44 = 0xfffffffffffull, M42 = 0x3ffffffffffull;
  uint64_t h0 = p->h0, h1 = p->h1, h2 = p->h2, c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  /* g = h + 5 - 2^130; take g if it did not borrow (h >= p) */
  uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
  uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
  uint64_t g2 = h2 + c - (1ull << 42);
  uint64_t mask = (g2 >> 63) - 1; /* all-ones if no borrow */
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  uint64_t lo = h0 | (h1 << 44), hi = (h1 >> 20) | (h2 << 24);
  u128 t = (u128)lo + p->pad0;
  lo = (uint64_t)t;
  hi = hi + p->pad1 + (uint64_t)(t >> 64);
  st64(tag, lo);
  st64(tag + 8, hi);
}

static void noise_nonce(uint64_t n, uint8_t nonce[12]) {
  memset(nonce, 0, 4); /* noise.cpp:207-215 */
  st64(nonce + 4, n);
}

/* keystream XOR for data blocks, counter starting at 1 (monocypher.c:2904) */
static void chacha_xor(const uint8_t key[32], const uint8_t nonce[12],
                       const uint8_t *in, uint8_t *out, size_t len) {
  uint8_t ks[64];
  for (uint32_t blk = 1; len; ++blk) {
    size_t n = len < 64 ? len : 64;
    oracle_chacha20_block(key, blk, nonce, ks);
    for (size_t i = 0; i < n; ++i) out[i] = in[i] ^ ks[i];
    in += n; out += n; len -= n;
  }
}

static void aead_tag(const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t *ad, size_t ad_len, const uint8_t *ct,
                     size_t len, uint8_t tag[16]) {
  uint8_t otk[64], sizes[16];
  poly_t p;
  oracle_chacha20_block(key, 0, nonce, otk); /* one-time key: block 0 */
  poly_init(&p, otk);
  poly_padded(&p, ad, ad_len);
  poly_padded(&p, ct, len);
  st64(sizes, ad_len);
  st64(sizes + 8, len);
  poly_block(&p, sizes);
  poly_final(&p, tag);
}

/* ENCRYPT(k, n, ad, pt): out[0..len) = ct, out[len..len+16) = tag.
 * in and out may alias exactly (in-place, as noise::encrypt does). */
void oracle_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                          size_t ad_len, const uint8_t *pt, size_t len,
                          uint8_t *out) {
  uint8_t nonce[12];
  noise_nonce(n, nonce);
  chacha_xor(key, nonce, pt, out, len);
  aead_tag(key, nonce, ad, ad_len, out, len, out + len);
}

/* DECRYPT(k, n, ad, ct||tag), ct_len includes the 16-byte tag.  Returns 0
 * and writes ct_len-16 plaintext bytes on success; returns -1 and leaves
 * `out` untouched on a MAC mismatch (crypto_aead_read, monocypher.c:2919-
 * 2926) or when ct_len < 16 (the reference's noise.cpp:257 underflows
 * there; the build defines it as an authentication failure). */
int oracle_noise_decrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                         size_t ad_len, const uint8_t *ct, size_t ct_len,
                         uint8_t *out) {
  if (ct_len < 16) return -1;
  size_t len = ct_len - 16;
  uint8_t nonce[12], tag[16], diff = 0;
  noise_nonce(n, nonce);
  aead_tag(key, nonce, ad, ad_len, ct, len, tag);
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ ct[len + i]);
  if (diff) return -1;
  chacha_xor(key, nonce, ct, out, len);
  return 0;
}

/* REKEY: k' = ENCRYPT(k, 2^64-2, empty, 0^32)[0..32)  (noise.cpp:429-439;
 * note 2^64-2, not the spec's 2^64-1). */
void oracle_rekey(const uint8_t key[32], uint8_t new_key[32]) {
  uint8_t buf[48] = {0};
  oracle_noise_encrypt(key, UINT64_MAX - 1, NULL, 0, buf, 32, buf);
  memcpy(new_key, buf, 32);
}

/* ---- synthetic record data (shared definition with the GPU generator in
 * noise-cpp_amd/csrc/noise_gpu.hip): byte j of a buffer is byte (j & 7) of
 * splitmix64 output number j >> 3, i.e. mix(seed + (i+1) * golden). */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t i) {
  return mix64(seed + (i + 1) * 0x9e3779b97f4a7c15ull);
}
void oracle_fill_synthetic(uint8_t *dst, uint64_t offset, uint64_t nbytes,
                           uint64_t seed) {
  for (uint64_t j = 0; j < nbytes; ++j) {
    uint64_t b = offset + j;
    dst[j] = (uint8_t)(oracle_splitmix64_at(seed, b >> 3) >> (8 * (b & 7)));
  }
}

/* ---- uniform batch helpers (parity tests at moderate sizes) ------------- */
typedef struct {
  const uint8_t *key;
  uint64_t n0;
  const uint8_t *in;
  size_t in_stride;
  uint8_t *out;
  size_t out_stride;
  size_t len;
  uint64_t lo, hi;
  int decrypt;
  int *status;
} job_t;

static void *run_job(void *arg) {
  job_t *j = (job_t *)arg;
  for (uint64_t r = j->lo; r < j->hi; ++r) {
    if (j->decrypt) {
      int rc = oracle_noise_decrypt(j->key, j->n0 + r, NULL, 0,
                                    j->in + r * j->in_stride, j->len + 16,
                                    j->out + r * j->out_stride);
      if (j->status) j->status[r] = rc;
    } else {
      oracle_noise_encrypt(j->key, j->n0 + r, NULL, 0,
                           j->in + r * j->in_stride, j->len,
                           j->out + r * j->out_stride);
    }
  }
  return NULL;
}

/* Encrypt (decrypt=0) or decrypt (decrypt=1) nrec uniform records with
 * nonces n0+i on `threads` pthreads.  Returns wall seconds. */
double oracle_batch_uniform(int decrypt, const uint8_t key[32], uint64_t n0,
                            const uint8_t *in, size_t in_stride, uint8_t *out,
                            size_t out_stride, size_t len, uint64_t nrec,
                            int threads, int *status) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  static pthread_t tid[1024];  /* one caller at a time (bench / tests) */
  static job_t jobs[1024];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    job_t j = {key, n0, in, in_stride, out, out_stride, len,
               nrec * t / threads, nrec * (t + 1) / threads, decrypt, status};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, run_job, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- whole-batch parity checkers (tests/: full-size configs) ------------
 * Every record of a batch the GPU processed is recomputed here and compared
 * byte for byte.  Descriptors use the C-ABI layout of noise_gpu_record
 * (include/noise_gpu.h: in_off, out_off, nonce, ad_off u64; len, ad_len,
 * key_idx, reserved u32 = 48 B), restated so this file needs no product
 * header.  `in` / `out` may be windows of larger buffers: a descriptor's
 * offset minus in_base / out_base indexes them (chunked device-to-host
 * copies).  Encrypt (decrypt = 0): out[out_off .. +len+16) must equal
 * ENCRYPT(key, nonce, ad, in[in_off .. +len)).  Decrypt (decrypt = 1):
 * status[i] must be 0 and out[out_off .. +len) the plaintext where the tag
 * verifies, 1 (NOISE_GPU_REC_BAD_MAC) where it does not, 2 for a key index
 * past the table or an all-zero key row (NOISE_GPU_REC_BAD_KEY).  Returns
 * the number of mismatching records; *first_bad receives the lowest index
 * of one (or -1). */
typedef struct {
  uint64_t in_off, out_off, nonce, ad_off;
  uint32_t len, ad_len, key_idx, reserved;
} oracle_rec_t;

typedef struct {
  int decrypt;
  const uint8_t *keys;
  uint32_t nkeys;
  const oracle_rec_t *recs;
  uint64_t in_base, out_base;
  const uint8_t *in, *ad;
  const uint8_t *out, *status;
  /* uniform form (recs == NULL): one key, nonce n0 + i, strided records */
  const uint8_t *key;
  uint64_t n0, in_stride, out_stride;
  uint32_t len;
  uint64_t lo, hi;
  int64_t bad, first;
} check_t;

static int zero_key(const uint8_t *k) {
  uint8_t acc = 0;
  for (int i = 0; i < 32; ++i) acc |= k[i];
  return acc == 0;
}

static void *run_check(void *arg) {
  check_t *c = (check_t *)arg;
  uint8_t *buf = NULL;
  size_t cap = 0;
  for (uint64_t i = c->lo; i < c->hi; ++i) {
    oracle_rec_t d;
    const uint8_t *key;
    if (c->recs) {
      d = c->recs[i];
      key = d.key_idx < c->nkeys ? c->keys + 32ull * d.key_idx : NULL;
    } else {
      d.in_off = i * c->in_stride;
      d.out_off = i * c->out_stride;
      d.nonce = c->n0 + i;
      d.ad_off = 0;
      d.len = c->len;
      d.ad_len = 0;
      key = c->key;
    }
    const uint8_t *in = c->in + (d.in_off - c->in_base);
    const uint8_t *out = c->out + (d.out_off - c->out_base);
    const uint8_t *ad = d.ad_len ? c->ad + d.ad_off : NULL;
    size_t need = (size_t)d.len + 16;
    if (need > cap) {
      free(buf);
      cap = need < 65552 ? 65552 : need;
      buf = (uint8_t *)malloc(cap);
    }
    int ok;
    if (!key || zero_key(key)) {
      /* encrypt: the GPU writes nothing for such a record (not checked
       * here); decrypt: status BAD_KEY */
      ok = !c->decrypt || c->status[i] == 2;
    } else if (!c->decrypt) {
      oracle_noise_encrypt(key, d.nonce, ad, d.ad_len, in, d.len, buf);
      ok = memcmp(buf, out, need) == 0;
    } else {
      int rc = oracle_noise_decrypt(key, d.nonce, ad, d.ad_len, in, need, buf);
      ok = rc == 0 ? (c->status[i] == 0 && memcmp(buf, out, d.len) == 0)
                   : c->status[i] == 1;
    }
    if (!ok) {
      if (c->first < 0) c->first = (int64_t)i;
      c->bad++;
    }
  }
  free(buf);
  return NULL;
}

static int64_t check_threads(check_t proto, uint64_t nrec, int threads, int64_t *first_bad) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if ((uint64_t)threads > nrec) threads = nrec ? (int)nrec : 1;
  pthread_t tid[256];
  check_t jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = proto;
    jobs[t].lo = nrec * t / threads;
    jobs[t].hi = nrec * (t + 1) / threads;
    jobs[t].bad = 0;
    jobs[t].first = -1;
    pthread_create(&tid[t], NULL, run_check, &jobs[t]);
  }
  int64_t bad = 0, first = -1;
  for (int t = 0; t < threads; ++t) {
    pthread_join(tid[t], NULL);
    bad += jobs[t].bad;
    if (jobs[t].first >= 0 && (first < 0 || jobs[t].first < first)) first = jobs[t].first;
  }
  if (first_bad) *first_bad = first;
  return bad;
}

/* descriptor batch on `threads` pthreads (bench.py cpu_baseline, "port"
 * kind when oracle/_ref is absent): 64-record chunks from a shared counter;
 * returns wall seconds, *fails = decrypt MAC failures */
typedef struct {
  int decrypt;
  const uint8_t *keys;
  const oracle_rec_t *recs;
  uint64_t nrec;
  const uint8_t *in;
  uint8_t *out;
  uint64_t *next;
  int fails;
} bjob_t;

static void *run_bjob(void *arg) {
  bjob_t *j = (bjob_t *)arg;
  for (;;) {
    const uint64_t lo = __atomic_fetch_add(j->next, 64, __ATOMIC_RELAXED);
    if (lo >= j->nrec) break;
    const uint64_t hi = lo + 64 < j->nrec ? lo + 64 : j->nrec;
    for (uint64_t i = lo; i < hi; ++i) {
      const oracle_rec_t *d = j->recs + i;
      const uint8_t *key = j->keys + 32ull * d->key_idx;
      if (j->decrypt)
        j->fails += oracle_noise_decrypt(key, d->nonce, NULL, 0, j->in + d->in_off,
                                         (size_t)d->len + 16, j->out + d->out_off) != 0;
      else
        oracle_noise_encrypt(key, d->nonce, NULL, 0, j->in + d->in_off, d->len,
                             j->out + d->out_off);
    }
  }
  return NULL;
}

double oracle_batch_records(int decrypt, const uint8_t *keys, const void *recs, uint64_t nrec,
                            const uint8_t *in, uint8_t *out, int threads, int *fails) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  static pthread_t tid[1024];
  static bjob_t jobs[1024];
  uint64_t next = 0;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    bjob_t j = {decrypt, keys, (const oracle_rec_t *)recs, nrec, in, out, &next, 0};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, run_bjob, &jobs[t]);
  }
  int f = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(tid[t], NULL);
    f += jobs[t].fails;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (fails) *fails = f;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

int64_t oracle_check_records(int decrypt, const uint8_t *keys, uint32_t nkeys,
                             const void *recs, uint64_t nrec, uint64_t in_base,
                             const uint8_t *in, uint64_t out_base, const uint8_t *out,
                             const uint8_t *ad, const uint8_t *status, int threads,
                             int64_t *first_bad) {
  check_t c;
  memset(&c, 0, sizeof c);
  c.decrypt = decrypt;
  c.keys = keys;
  c.nkeys = nkeys;
  c.recs = (const oracle_rec_t *)recs;
  c.in_base = in_base;
  c.out_base = out_base;
  c.in = in;
  c.out = out;
  c.ad = ad;
  c.status = status;
  return check_threads(c, nrec, threads, first_bad);
}

/* uniform form: record i at in + i * in_stride / out + i * out_stride, nonce
 * n0 + i, one key, no AD (status indexed from 0 like the records) */
int64_t oracle_check_uniform(int decrypt, const uint8_t key[32], uint64_t n0,
                             const uint8_t *in, uint64_t in_stride, const uint8_t *out,
                             uint64_t out_stride, uint32_t len, uint64_t nrec,
                             const uint8_t *status, int threads, int64_t *first_bad) {
  check_t c;
  memset(&c, 0, sizeof c);
  c.decrypt = decrypt;
  c.key = key;
  c.n0 = n0;
  c.in = in;
  c.out = out;
  c.in_stride = in_stride;
  c.out_stride = out_stride;
  c.len = len;
  c.status = status;
  return check_threads(c, nrec, threads, first_bad);
}
