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
