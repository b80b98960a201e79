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
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job_t jobs[256];
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
