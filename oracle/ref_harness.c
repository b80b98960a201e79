/*
 * oracle/ref_harness.c -- calls the REFERENCE's own Monocypher AEAD with
 * the reference's Noise nonce framing.  TEST/BASELINE INFRASTRUCTURE ONLY.
 *
 * Built by oracle/Makefile together with /root/reference/monocypher.c
 * (compiled as-is from where it lies; never copied) into
 * oracle/_ref/libnoise_ref.so.  It restates only the framing of
 * noise::encrypt / noise::decrypt (noise.cpp:202-224, 254-281): nonce =
 * 0^32 || LE64(n), crypto_aead_init_ietf + crypto_aead_write/_read.
 * noise.cpp itself is not built: it needs <format>, which this image's
 * libstdc++ (GCC 11) lacks, and stand-in headers are not allowed.
 *
 * Used (a) by tests/test_oracle.py to pin oracle/chachapoly_oracle.c against
 * monocypher, and (b) by bench.py's cpu_baseline leg (kind "reference").
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "monocypher.h"

static void nonce_of(uint64_t n, uint8_t nonce[12]) {
  memset(nonce, 0, 12);
  for (int i = 0; i < 8; ++i) nonce[4 + i] = (uint8_t)(n >> (8 * i));
}

void ref_noise_encrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                       size_t ad_len, const uint8_t *pt, size_t len,
                       uint8_t *out) {
  uint8_t nonce[12];
  crypto_aead_ctx ctx;
  nonce_of(n, nonce);
  crypto_aead_init_ietf(&ctx, key, nonce);
  crypto_aead_write(&ctx, out, out + len, ad, ad_len, pt, len);
  crypto_wipe(&ctx, sizeof ctx);
}

int ref_noise_decrypt(const uint8_t key[32], uint64_t n, const uint8_t *ad,
                      size_t ad_len, const uint8_t *ct, size_t ct_len,
                      uint8_t *out) {
  uint8_t nonce[12];
  crypto_aead_ctx ctx;
  if (ct_len < 16) return -1;
  nonce_of(n, nonce);
  crypto_aead_init_ietf(&ctx, key, nonce);
  int rc = crypto_aead_read(&ctx, out, ct + ct_len - 16, ad, ad_len, ct,
                            ct_len - 16);
  crypto_wipe(&ctx, sizeof ctx);
  return rc;
}

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
  int fails;
} job_t;

static void *run_job(void *arg) {
  job_t *j = (job_t *)arg;
  for (uint64_t r = j->lo; r < j->hi; ++r) {
    if (j->decrypt)
      j->fails += ref_noise_decrypt(j->key, j->n0 + r, NULL, 0,
                                    j->in + r * j->in_stride, j->len + 16,
                                    j->out + r * j->out_stride) != 0;
    else
      ref_noise_encrypt(j->key, j->n0 + r, NULL, 0, j->in + r * j->in_stride,
                        j->len, j->out + r * j->out_stride);
  }
  return NULL;
}

/* Uniform batch through monocypher on `threads` pthreads; returns wall
 * seconds, *fails = number of MAC failures (decrypt). */
double ref_batch_uniform(int decrypt, const uint8_t key[32], uint64_t n0,
                         const uint8_t *in, size_t in_stride, uint8_t *out,
                         size_t out_stride, size_t len, uint64_t nrec,
                         int threads, int *fails) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  static pthread_t tid[1024];
  static job_t jobs[1024];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    job_t j = {key, n0, in, in_stride, out, out_stride, len,
               nrec * t / threads, nrec * (t + 1) / threads, decrypt, 0};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, run_job, &jobs[t]);
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

/* ---- descriptor batches (BASELINE configs 3 and 4 on the CPU) ------------
 * Records in the C-ABI descriptor layout (include/noise_gpu.h
 * noise_gpu_record: in_off, out_off, nonce, ad_off u64; len, ad_len, key_idx,
 * reserved u32), restated here; no AD.  Each record is one noise::encrypt /
 * noise::decrypt call (crypto_aead_init_ietf + crypto_aead_write/_read with
 * the Noise nonce), exactly what CipherState::encrypt_with_ad does per
 * record.  Threads take 64-record chunks from a shared counter, so mixed
 * sizes balance. */
typedef struct {
  uint64_t in_off, out_off, nonce, ad_off;
  uint32_t len, ad_len, key_idx, reserved;
} ref_rec_t;

typedef struct {
  int decrypt;
  const uint8_t *keys;
  const ref_rec_t *recs;
  uint64_t nrec;
  const uint8_t *in;
  uint8_t *out;
  uint64_t *next;
  int fails;
} rjob_t;

static void *run_rjob(void *arg) {
  rjob_t *j = (rjob_t *)arg;
  for (;;) {
    const uint64_t lo = __atomic_fetch_add(j->next, 64, __ATOMIC_RELAXED);
    if (lo >= j->nrec) break;
    const uint64_t hi = lo + 64 < j->nrec ? lo + 64 : j->nrec;
    for (uint64_t i = lo; i < hi; ++i) {
      const ref_rec_t *d = j->recs + i;
      const uint8_t *key = j->keys + 32ull * d->key_idx;
      if (j->decrypt)
        j->fails += ref_noise_decrypt(key, d->nonce, NULL, 0, j->in + d->in_off,
                                      (size_t)d->len + 16, j->out + d->out_off) != 0;
      else
        ref_noise_encrypt(key, d->nonce, NULL, 0, j->in + d->in_off, d->len,
                          j->out + d->out_off);
    }
  }
  return NULL;
}

double ref_batch_records(int decrypt, const uint8_t *keys, const void *recs, uint64_t nrec,
                         const uint8_t *in, uint8_t *out, int threads, int *fails) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  static pthread_t tid[1024];
  static rjob_t jobs[1024];
  uint64_t next = 0;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    rjob_t j = {decrypt, keys, (const ref_rec_t *)recs, nrec, in, out, &next, 0};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, run_rjob, &jobs[t]);
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

/* The reference's X25519 (monocypher.c:1546-1563, called by noise::dh,
 * noise.cpp:172-177): one result, for parity, and a timed loop on `threads`
 * host threads for the CPU baseline of tools/bench_x25519.py.  Returns the
 * wall seconds of n scalar multiplications (chained: each output is the
 * next point, so nothing is skipped). */
void ref_x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
  crypto_x25519(out, scalar, point);
}

struct xjob {
  uint8_t k[32], u[32];
  long n;
};

static void *run_x(void *arg) {
  struct xjob *j = (struct xjob *)arg;
  for (long i = 0; i < j->n; ++i) crypto_x25519(j->u, j->k, j->u);
  return NULL;
}

double ref_x25519_bench(long n, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t th[64];
  struct xjob jobs[64];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    for (int b = 0; b < 32; ++b) {
      jobs[t].k[b] = (uint8_t)(7 * b + t + 1);
      jobs[t].u[b] = (uint8_t)(b == 0 ? 9 : 0);
    }
    jobs[t].n = n / threads;
    pthread_create(&th[t], NULL, run_x, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- Noise_XX_25519_ChaChaPoly_BLAKE2b on the reference's primitives ----
 * Both parties of one XX handshake (rev34 §5.2-5.3, §7.5), composed from
 * Monocypher's crypto_blake2b / crypto_x25519 / AEAD exactly as noise.cpp's
 * hash / hmac_hash / hkdf / dh / encrypt (noise.cpp:172-374) compose them,
 * with the spec's HasKey() (the reference's is inverted).  Empty
 * prologue and payloads.  Used (a) by tests to pin the batched GPU handshake
 * (noise_gpu_hs_*) on random keys against the reference's own primitives,
 * (b) as the CPU baseline of tools/bench_handshake.py. */
typedef struct {
  uint8_t ck[64], h[64], k[32];
  int has_k;
  uint64_t n;
} sym_t;

static void hmac_b2(const uint8_t key[64], const uint8_t *d1, size_t l1, const uint8_t *d2,
                    size_t l2, uint8_t out[64]) {
  uint8_t blk[128], inner[64];
  crypto_blake2b_ctx c;
  for (int i = 0; i < 128; ++i) blk[i] = (uint8_t)((i < 64 ? key[i] : 0) ^ 0x36);
  crypto_blake2b_init(&c, 64);
  crypto_blake2b_update(&c, blk, 128);
  crypto_blake2b_update(&c, d1, l1);
  crypto_blake2b_update(&c, d2, l2);
  crypto_blake2b_final(&c, inner);
  for (int i = 0; i < 128; ++i) blk[i] = (uint8_t)((i < 64 ? key[i] : 0) ^ 0x5c);
  crypto_blake2b_init(&c, 64);
  crypto_blake2b_update(&c, blk, 128);
  crypto_blake2b_update(&c, inner, 64);
  crypto_blake2b_final(&c, out);
  crypto_wipe(blk, sizeof blk);
  crypto_wipe(inner, sizeof inner);
}

static void hkdf_b2(const uint8_t ck[64], const uint8_t *ikm, size_t ilen, uint8_t o1[64],
                    uint8_t o2[64]) {
  uint8_t tk[64], one = 1, two = 2;
  hmac_b2(ck, ikm, ilen, NULL, 0, tk);
  hmac_b2(tk, &one, 1, NULL, 0, o1);
  hmac_b2(tk, o1, 64, &two, 1, o2);
  crypto_wipe(tk, sizeof tk);
}

static void sym_mix_hash(sym_t *s, const uint8_t *d, size_t len) {
  crypto_blake2b_ctx c;
  crypto_blake2b_init(&c, 64);
  crypto_blake2b_update(&c, s->h, 64);
  crypto_blake2b_update(&c, d, len);
  crypto_blake2b_final(&c, s->h);
}

static void sym_mix_key(sym_t *s, const uint8_t ikm[32]) {
  uint8_t o1[64], o2[64];
  hkdf_b2(s->ck, ikm, 32, o1, o2);
  memcpy(s->ck, o1, 64);
  memcpy(s->k, o2, 32);
  s->has_k = 1;
  s->n = 0;
}

static void sym_dh(sym_t *s, const uint8_t sk[32], const uint8_t pk[32]) {
  uint8_t shared[32];
  crypto_x25519(shared, sk, pk);
  sym_mix_key(s, shared);
  crypto_wipe(shared, 32);
}

/* out = ct (len + 16 when keyed) */
static size_t sym_encrypt_hash(sym_t *s, const uint8_t *pt, size_t len, uint8_t *out) {
  size_t olen = len;
  if (s->has_k) {
    ref_noise_encrypt(s->k, s->n++, s->h, 64, pt, len, out);
    olen += 16;
  } else {
    memcpy(out, pt, len);
  }
  sym_mix_hash(s, out, olen);
  return olen;
}

static int sym_decrypt_hash(sym_t *s, const uint8_t *ct, size_t ct_len, uint8_t *out) {
  int rc = 0;
  if (s->has_k) rc = ref_noise_decrypt(s->k, s->n++, s->h, 64, ct, ct_len, out);
  else memcpy(out, ct, ct_len);
  sym_mix_hash(s, ct, ct_len);
  return rc;
}

static void sym_init(sym_t *s) {
  static const char name[] = "Noise_XX_25519_ChaChaPoly_BLAKE2b";
  memset(s, 0, sizeof *s);
  memcpy(s->h, name, sizeof name - 1);  /* <= 64 bytes: padded, not hashed */
  memcpy(s->ck, s->h, 64);
  sym_mix_hash(s, NULL, 0);             /* MixHash(empty prologue) */
}

int ref_xx_handshake(const uint8_t si[32], const uint8_t ei[32], const uint8_t sr[32],
                     const uint8_t er[32], uint8_t msgs[192], uint8_t hash[64], uint8_t k1[32],
                     uint8_t k2[32]) {
  sym_t I, R;
  uint8_t spk_i[32], spk_r[32], epk_i[32], epk_r[32], rs_i[48], rs_r[48], tmp[48];
  uint8_t *m1 = msgs, *m2 = msgs + 32, *m3 = msgs + 128;
  int rc = 0;
  crypto_x25519_public_key(spk_i, si);
  crypto_x25519_public_key(spk_r, sr);
  sym_init(&I);
  sym_init(&R);
  /* -> e */
  crypto_x25519_public_key(epk_i, ei);
  memcpy(m1, epk_i, 32);
  sym_mix_hash(&I, epk_i, 32);
  sym_encrypt_hash(&I, NULL, 0, tmp);
  sym_mix_hash(&R, m1, 32);
  rc |= sym_decrypt_hash(&R, NULL, 0, tmp);
  /* <- e, ee, s, es */
  crypto_x25519_public_key(epk_r, er);
  memcpy(m2, epk_r, 32);
  sym_mix_hash(&R, epk_r, 32);
  sym_dh(&R, er, m1);
  sym_encrypt_hash(&R, spk_r, 32, m2 + 32);
  sym_dh(&R, sr, m1);
  sym_encrypt_hash(&R, NULL, 0, m2 + 80);
  sym_mix_hash(&I, m2, 32);
  sym_dh(&I, ei, m2);
  rc |= sym_decrypt_hash(&I, m2 + 32, 48, rs_i);
  sym_dh(&I, ei, rs_i);
  rc |= sym_decrypt_hash(&I, m2 + 80, 16, tmp);
  /* -> s, se */
  sym_encrypt_hash(&I, spk_i, 32, m3);
  sym_dh(&I, si, m2);
  sym_encrypt_hash(&I, NULL, 0, m3 + 48);
  rc |= sym_decrypt_hash(&R, m3, 48, rs_r);
  sym_dh(&R, er, rs_r);
  rc |= sym_decrypt_hash(&R, m3 + 48, 16, tmp);
  /* Split (both sides agree when rc == 0) */
  uint8_t o1[64], o2[64];
  hkdf_b2(I.ck, NULL, 0, o1, o2);
  memcpy(k1, o1, 32);
  memcpy(k2, o2, 32);
  memcpy(hash, I.h, 64);
  if (memcmp(I.h, R.h, 64) != 0 || memcmp(I.ck, R.ck, 64) != 0) rc = -1;
  crypto_wipe(&I, sizeof I);
  crypto_wipe(&R, sizeof R);
  crypto_wipe(o1, 64);
  crypto_wipe(o2, 64);
  return rc ? -1 : 0;
}

struct hjob {
  long n;
  int seed, fails;
};

static void *run_h(void *arg) {
  struct hjob *j = (struct hjob *)arg;
  uint8_t si[32], sr[32], ei[32], er[32], msgs[192], hash[64], k1[32], k2[32];
  for (int b = 0; b < 32; ++b) {
    si[b] = (uint8_t)(3 * b + j->seed);
    sr[b] = (uint8_t)(5 * b + j->seed);
  }
  for (long i = 0; i < j->n; ++i) {
    for (int b = 0; b < 32; ++b) {  /* fresh ephemerals per handshake */
      ei[b] = (uint8_t)(b + i + j->seed);
      er[b] = (uint8_t)(7 * b + i);
    }
    j->fails += ref_xx_handshake(si, ei, sr, er, msgs, hash, k1, k2) != 0;
  }
  return NULL;
}

/* n full XX handshakes (both parties, as the GPU bench counts them) on
 * `threads` pthreads; wall seconds, *fails = handshakes that did not agree. */
double ref_xx_bench(long n, int threads, int *fails) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t th[64];
  struct hjob jobs[64];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; ++t) {
    jobs[t].n = n / threads;
    jobs[t].seed = t + 1;
    jobs[t].fails = 0;
    pthread_create(&th[t], NULL, run_h, &jobs[t]);
  }
  int f = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    f += jobs[t].fails;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (fails) *fails = f;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
