/*
 * noise_gpu.h -- C ABI of the MI355X (gfx950) Noise transport-record AEAD
 * engine (ChaChaPoly, Noise nonce framing).
 *
 * This is the drop-in boundary under noise::CipherState.  In the reference
 * (ethindp/noise-cpp @ 2025-09-05) every transport record goes
 *     CipherState::encrypt_with_ad / decrypt_with_ad   noise.cpp:393-427
 *  -> noise::encrypt / noise::decrypt                   noise.cpp:202-281
 *  -> crypto_aead_init_ietf + crypto_aead_write/_read    monocypher.c:2891-2929
 * and CipherState::rekey (noise.cpp:429-439) calls noise::encrypt at nonce
 * 2^64-2.  The functions below replace that chain: the C++20 CipherState in
 * noise-cpp_amd/host/ (same class surface as noise.h:99-115) calls them,
 * and device-resident batch callers may call them directly.
 *
 * Conventions
 *  - Plain pointers and sizes only.  `d_` pointers are device (HBM)
 *    pointers, `h_` pointers host pointers.  `stream` is a hipStream_t
 *    passed as void* (NULL = the legacy default stream).
 *  - Device-pointer functions are asynchronous on `stream`: argument
 *    checks happen at the call, results are ready when the stream is.
 *  - No function throws; every function returns a noise_gpu_status.
 *  - Record i of a uniform batch uses nonce (nonce0 + i) mod 2^64, the
 *    Noise 12-byte nonce 0^32 || LE64(n) (noise.cpp:207-215).
 *  - Ciphertext records are the Noise wire format ct || tag: len+16 bytes.
 *  - Nonce-limit (noise.cpp:398-400, 416-418: n == 2^64-2 is refused) is a
 *    host-object rule; the batch functions below encrypt whatever nonces
 *    they are given.  The CipherState shim applies the rule per record.
 */
#ifndef NOISE_GPU_H
#define NOISE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum noise_gpu_status {
  NOISE_GPU_OK = 0,
  NOISE_GPU_E_NONCE = 1, /* nonce limit; reference std::out_of_range      */
  NOISE_GPU_E_MAC = 2,   /* tag mismatch; reference std::invalid_argument */
  NOISE_GPU_E_ARG = 3,   /* bad argument (null, size, alignment, range)   */
  NOISE_GPU_E_HIP = 4,   /* HIP runtime error (see noise_gpu_last_error)  */
  NOISE_GPU_E_NODEV = 5  /* no gfx950 device visible                      */
} noise_gpu_status;

/* Per-record descriptor for many-session / variable-length batches.
 * Offsets are byte offsets into the d_in / d_out / d_ad buffers. */
typedef struct noise_gpu_record {
  uint64_t in_off;  /* plaintext (encrypt) or ct||tag (decrypt) */
  uint64_t out_off; /* ct||tag (encrypt) or plaintext (decrypt)  */
  uint64_t nonce;   /* Noise n for this record                   */
  uint64_t ad_off;  /* associated data offset (ignored if ad_len == 0) */
  uint32_t len;     /* plaintext length, <= 65519 for Noise messages */
  uint32_t ad_len;  /* associated data length                    */
  uint32_t key_idx; /* row of the [nkeys][32] key table          */
  uint32_t reserved;
} noise_gpu_record;

/* Per-record status codes written by the decrypt functions. */
#define NOISE_GPU_REC_OK 0u
#define NOISE_GPU_REC_BAD_MAC 1u

/* ---- runtime ---------------------------------------------------------- */

/* Version string of the engine ("noise-mi355x <ver> gfx950"). */
const char *noise_gpu_version(void);
/* Human-readable text of a status code. */
const char *noise_gpu_strerror(int status);
/* Text of the last HIP error seen by this thread (empty if none). */
const char *noise_gpu_last_error(void);
/* Number of visible HIP devices (0 without a GPU). */
int noise_gpu_device_count(int *count);

/* ---- device-resident uniform batches (the BASELINE hot path) -----------
 * nrec records of exactly `len` plaintext bytes under one 32-byte key (an
 * all-zero key is "no key", Noise HasKey() false, and is refused with
 * NOISE_GPU_E_ARG rather than used as a publicly known key).
 * Record i: input at d_in + i*in_stride, output at d_out + i*out_stride,
 * associated data at d_ad + i*ad_stride (ad_stride 0 = the same AD for every
 * record; ad_len 0 = no AD, the transport case).
 * Encrypt writes len+16 bytes per record (ct || tag).  in == out with equal
 * strides is in-place; other overlaps are undefined.
 * Decrypt reads len+16 bytes per record, writes len plaintext bytes only
 * where the tag verifies (both the tile kernel and the one-lane-per-record
 * path check the tag before storing any plaintext), and writes d_status[i]
 * (NOISE_GPU_REC_*).  A
 * record whose tag fails is left as it was when in-place (the reference
 * leaves the buffer untouched, monocypher.c:2919-2926) and is zeroed in an
 * out-of-place output (no unauthenticated plaintext is left behind).
 * 16-byte aligned pointers/strides, ad_len == 0 and len in {64, 128, 192,
 * 256, 512, 1024, 2048, 4096, 8192, 16384} run on the LDS-staged tile kernel
 * (the hot path); any other len of 1..16384 with 16-byte aligned pointers
 * and strides and no AD on the masked tile kernel, at the smallest tile
 * capacity >= len (the powers of two above and 320, 384, 448, 768, 1280,
 * 1536, 1792, 2304, 2560, 3072, 5120); unaligned records (strides or bases
 * not multiples of 16) of len <= 16384 without AD, in batches of >= 1024
 * records that do not partially overlap, are copied into an aligned image in
 * the library's scratch for (device, stream) (noise_gpu_scratch_wipe clears
 * it), processed there and copied back; other shapes (AD, len > 16384, small
 * unaligned batches) one record per lane (vector path when 16-byte aligned
 * with len % 16 == 0, byte-granular otherwise).
 * Key handling: h_key is copied into the kernel's argument block (kernarg
 * memory) by value, so the 32-byte key stays in that launch's kernarg
 * segment after the call, like any kernel argument; the runtime reuses,
 * but does not wipe, kernarg memory.  Callers that must not leave a key
 * there use the sessions / descriptor functions, whose keys live in a
 * device key table the caller owns and wipes. */
int noise_gpu_encrypt_uniform(const uint8_t h_key[32], uint64_t nonce0,
                              const uint8_t *d_in, uint64_t in_stride,
                              uint8_t *d_out, uint64_t out_stride,
                              uint32_t len, const uint8_t *d_ad,
                              uint64_t ad_stride, uint32_t ad_len,
                              uint64_t nrec, void *stream);

int noise_gpu_decrypt_uniform(const uint8_t h_key[32], uint64_t nonce0,
                              const uint8_t *d_in, uint64_t in_stride,
                              uint8_t *d_out, uint64_t out_stride,
                              uint32_t len, const uint8_t *d_ad,
                              uint64_t ad_stride, uint32_t ad_len,
                              uint8_t *d_status, uint64_t nrec, void *stream);

/* ---- device-resident descriptor batches (many sessions, mixed sizes) ---
 * d_keys: [nkeys][32] key table in HBM (16-byte aligned); d_recs: nrec
 * descriptors in HBM.  Same in-place / failure rules as the uniform
 * functions; a record is in place when d_in + in_off == d_out + out_off.
 * A descriptor whose key_idx >= nkeys, or whose key row is all zero (the
 * "no key" row noise_gpu_hs_split gives a failed handshake), is not processed
 * (nothing written; decrypt status NOISE_GPU_REC_BAD_KEY).
 * Batches of >= 2048 records are load-balanced on the device, stream-ordered
 * (no host synchronisation): records are sorted by class and each class
 * runs its own kernel -- 16-byte aligned AD-free records of any length up to
 * 2048 bytes, and of exactly 4096, 8192 and 16384, on the LDS-staged
 * masked tile kernel, one launch per tile capacity (64, 128, 192, 256,
 * 512 B, 1, 2, 4, 8, 16 KiB: the smallest that holds the record; a record
 * sits whole in one wave, and decrypt reads its ciphertext once); the other
 * aligned AD-free records of 2049..65535 bytes cut into
 * 1 KiB segments that ONE tile-kernel launch processes, plus their tails
 * (len % 1024, masked 1 KiB tile units) and a per-record finalize (tag);
 * everything else one lane per record.  Every path checks a record's
 * tag before any of its plaintext is stored (crypto_aead_read,
 * monocypher.c:2912-2929): the tile classes and the one-lane-per-record path
 * per record; a segmented (>= 1 KiB) record by a Poly1305 pass over its
 * ciphertext and the finalize's tag check, after which a keystream pass
 * writes the plaintext of the records that verified -- the output range of a
 * failed record never holds a byte of its plaintext, not even transiently.
 * Scratch is a grow-only device buffer per (device, stream).  The classes
 * run on three companion streams the library creates per (device, stream)
 * and joins back with events (no host synchronisation); with the caller's
 * stream that is four HIP streams, the runtime's default number of hardware
 * queues per process (GPU_MAX_HW_QUEUES = 4): further streams of the caller's
 * own share those queues with them. */
int noise_gpu_encrypt_records(const uint8_t *d_keys, uint32_t nkeys,
                              const noise_gpu_record *d_recs, uint64_t nrec,
                              const uint8_t *d_in, uint8_t *d_out,
                              const uint8_t *d_ad, void *stream);

int noise_gpu_decrypt_records(const uint8_t *d_keys, uint32_t nkeys,
                              const noise_gpu_record *d_recs, uint64_t nrec,
                              const uint8_t *d_in, uint8_t *d_out,
                              const uint8_t *d_ad, uint8_t *d_status,
                              void *stream);

/* The same, with len_sum = the sum of the descriptors' len (0 = unknown).
 * Below 2048 records the plain functions run ONE lane per record, which is
 * fastest for short records but walks a long one serially (~19 us per KiB);
 * with len_sum given, a batch whose records average >= 2 KiB takes the
 * load-balanced path instead (100 x 16 KiB: 0.35 ms instead of 1.9 ms per
 * encrypt + decrypt pair).  Used by noise::transport::Pipeline; the
 * host-buffer records functions compute it themselves. */
int noise_gpu_encrypt_records_sized(const uint8_t *d_keys, uint32_t nkeys,
                                    const noise_gpu_record *d_recs, uint64_t nrec,
                                    const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_ad,
                                    uint64_t len_sum, void *stream);
int noise_gpu_decrypt_records_sized(const uint8_t *d_keys, uint32_t nkeys,
                                    const noise_gpu_record *d_recs, uint64_t nrec,
                                    const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_ad,
                                    uint8_t *d_status, uint64_t len_sum, void *stream);

/* The descriptor path keeps a grow-only device scratch per (device,
 * stream) that holds, between the kernels of a call, copies of the long
 * records' keys, their one-time Poly1305 keys and partial sums.  This zeroes
 * it (stream-ordered after the calls already issued on `stream`), e.g. at
 * session teardown.  The host-buffer entry points below wipe it themselves. */
int noise_gpu_scratch_wipe(void *stream);

/* Zero and free the records scratch and the companion stream the descriptor
 * path cached for (current device, `stream`); synchronises `stream` first.
 * Call it before destroying a stream of your own that the descriptor
 * functions were called on (noise_gpu_ctx_destroy does it for the context's
 * streams); otherwise both stay allocated until the library is unloaded.
 * A stream with nothing cached is a no-op. */
int noise_gpu_scratch_release(void *stream);

/* ---- device-resident many-session batches (BASELINE config 3) ---------
 * nrec records of `len` plaintext bytes, record i under key row
 * d_keys[d_key_idx[i]] (a [nkeys][32] table, 16-byte aligned) with Noise
 * nonce d_nonces[i]; records laid out like the uniform batches (d_in + i *
 * in_stride, d_out + i * out_stride).  No associated data (transport).
 * Served by the LDS-staged tile kernel: len in {64, 128, 192, 256, 512,
 * 1024, 2048, 4096, 8192, 16384} with 16-byte aligned buffers/strides; other shapes
 * return NOISE_GPU_E_ARG (use the descriptor functions below).  A record
 * whose key index is >= nkeys, or whose key row is all zero, is not written;
 * decrypt marks it NOISE_GPU_REC_BAD_KEY.  Tags are checked before any
 * plaintext is stored. */
#define NOISE_GPU_REC_BAD_KEY 2u
int noise_gpu_encrypt_sessions(const uint8_t *d_keys, uint32_t nkeys,
                               const uint32_t *d_key_idx,
                               const uint64_t *d_nonces, const uint8_t *d_in,
                               uint64_t in_stride, uint8_t *d_out,
                               uint64_t out_stride, uint32_t len, uint64_t nrec,
                               void *stream);
int noise_gpu_decrypt_sessions(const uint8_t *d_keys, uint32_t nkeys,
                               const uint32_t *d_key_idx,
                               const uint64_t *d_nonces, const uint8_t *d_in,
                               uint64_t in_stride, uint8_t *d_out,
                               uint64_t out_stride, uint32_t len,
                               uint8_t *d_status, uint64_t nrec, void *stream);

/* REKEY of every key in a device key table, in place:
 * k <- ENCRYPT(k, 2^64-2, empty, 0^32)[0..32)   (noise.cpp:429-439). */
int noise_gpu_rekey_keys(uint8_t *d_keys, uint64_t nkeys, void *stream);

/* ---- batched X25519 (mass handshakes) -----------------------------------
 * d_out[i] = X25519(d_scalars[i], d_points[i]) for i < n: 32-byte little-
 * endian scalars (clamped as RFC 7748 §5), u-coordinates and results, 16-byte
 * aligned arrays of n x 32 bytes.  d_points == NULL: the base point u = 9
 * (public keys).  Replaces, for many sessions at once, noise::dh /
 * generate_keypair -> crypto_x25519 / crypto_x25519_public_key
 * (noise.cpp:164-177, monocypher.c:1546-1563).  Asynchronous on stream. */
int noise_gpu_x25519(const uint8_t *d_scalars, const uint8_t *d_points,
                     uint8_t *d_out, uint64_t n, void *stream);

/* ---- batched handshakes (mass handshakes) -------------------------------
 * n sessions running the same pattern in the same role, in lockstep: every
 * token of a message runs as one GPU kernel over all n sessions (one lane per
 * session: X25519 ladder, BLAKE2b / HMAC / HKDF, ChaChaPoly with AD = h),
 * session state resident in HBM.  Replaces, for many handshakes at once,
 * noise::HandshakeState initialize / write_message / read_message / finalize
 * (noise.h:137-173, noise.cpp:545-1100), with the spec semantics of the host
 * noise::HandshakeState (noise_amd/handshake.hpp; suite
 * Noise_<pattern>_25519_ChaChaPoly_BLAKE2b).  All functions are asynchronous
 * on `stream` except create/destroy/info; arrays are device pointers.
 *
 * Per-session byte ranges are described by a span: session i's bytes start
 * at base + (off ? off[i] : i * stride) and are len ? len[i] : len_all long
 * (the length is ignored where the library determines it). */
typedef struct noise_gpu_span {
  uint8_t *base;
  const uint64_t *off; /* per-session offsets, or NULL: i * stride      */
  uint64_t stride;
  const uint32_t *len; /* per-session lengths, or NULL: len_all         */
  uint32_t len_all;
  uint32_t reserved;
} noise_gpu_span;

typedef struct noise_gpu_hs noise_gpu_hs;

/* key slots of noise_gpu_hs_set_key */
#define NOISE_GPU_HS_S 0  /* local static private key (public derived)  */
#define NOISE_GPU_HS_E 1  /* local ephemeral private key (test vectors;
                             otherwise generated at the "e" token)       */
#define NOISE_GPU_HS_RS 2 /* remote static public key                   */
#define NOISE_GPU_HS_RE 3 /* remote ephemeral public key                */

/* per-session status (noise_gpu_hs_status, read_message) */
#define NOISE_GPU_HS_OK 0u
#define NOISE_GPU_HS_BAD_MAC 1u /* a handshake AEAD tag did not verify */
#define NOISE_GPU_HS_BAD_LEN 3u /* message shorter than its tokens, or > 65535 */

typedef struct noise_gpu_hs_info {
  uint32_t message_index; /* next message of the pattern (0-based)         */
  uint32_t message_count;
  int32_t my_turn;        /* 1: next call is write_message, 0: read_message */
  int32_t finished;       /* all messages done: split() may be called     */
  uint32_t overhead;      /* bytes of the next message besides the payload
                             (token bytes + the payload tag if keyed)     */
  uint32_t psk_count;     /* psks each session needs (noise_gpu_hs_set_psks) */
} noise_gpu_hs_info;

/* pattern: name as in the protocol name, with psk modifiers ("XX", "IK",
 * "XXpsk0+psk2").  n: sessions.  Allocates n x 384 B of device state on the
 * current device. */
int noise_gpu_hs_create(const char *pattern, int initiator, uint64_t n,
                        noise_gpu_hs **out);
/* wipes the device state, then frees it (synchronises the device) */
int noise_gpu_hs_destroy(noise_gpu_hs *hs);
int noise_gpu_hs_info_get(const noise_gpu_hs *hs, noise_gpu_hs_info *out);
/* Before noise_gpu_hs_start: install key slot `which` for every session from
 * d_keys (32 bytes per session at `stride`; stride 0 = one key for all). */
int noise_gpu_hs_set_key(noise_gpu_hs *hs, int which, const uint8_t *d_keys,
                         uint64_t stride, void *stream);
/* Before noise_gpu_hs_start: the psks, n x psk_count x 32 bytes (copied). */
int noise_gpu_hs_set_psks(noise_gpu_hs *hs, const uint8_t *d_psks, void *stream);
/* InitializeSymmetric + MixHash(prologue) + the pre-messages.  prologue may
 * be NULL (empty prologue for every session). */
int noise_gpu_hs_start(noise_gpu_hs *hs, const noise_gpu_span *prologue,
                       void *stream);
/* WriteMessage for every session: payload (NULL = empty) -> msg at msg's
 * offsets (msg lengths ignored; each needs overhead + payload bytes);
 * d_msg_len (may be NULL) receives the message lengths. */
int noise_gpu_hs_write_message(noise_gpu_hs *hs, const noise_gpu_span *payload,
                               const noise_gpu_span *msg, uint32_t *d_msg_len,
                               void *stream);
/* ReadMessage for every session: msg (with lengths) -> payload at payload's
 * offsets (room for msg length - overhead bytes; may be NULL if every payload
 * is empty).  d_payload_len (may be NULL): payload lengths; d_status (may be
 * NULL): per-session NOISE_GPU_HS_* after this message.  A failed session
 * stays failed: later calls skip it and split() gives it all-zero keys. */
int noise_gpu_hs_read_message(noise_gpu_hs *hs, const noise_gpu_span *msg,
                              const noise_gpu_span *payload,
                              uint32_t *d_payload_len, uint8_t *d_status,
                              void *stream);
int noise_gpu_hs_status(const noise_gpu_hs *hs, uint8_t *d_status, void *stream);
/* Split() of every finished session: d_k1[i] (initiator -> responder) and
 * d_k2[i] (responder -> initiator), 32-byte key rows that the sessions /
 * records entry points take as key tables; optionally the handshake hash
 * (64-byte rows) and the remote static public key (32-byte rows). */
int noise_gpu_hs_split(noise_gpu_hs *hs, uint8_t *d_k1, uint8_t *d_k2,
                       uint8_t *d_hash, uint8_t *d_rs, void *stream);

/* ---- host-buffer entry points (synchronous) ----------------------------
 * Used by the CipherState shim for single records (encrypt_with_ad /
 * decrypt_with_ad / rekey).  A record of <= 65535 bytes with <= 8192 bytes of
 * AD runs as ONE kernel launch (256 threads) that reads and writes a
 * per-thread host-mapped pinned staging buffer directly (no copies, one
 * launch, completion seen by polling a done word the kernel writes last);
 * larger ones stage through pinned memory and a device buffer.  Either way
 * the tag is checked before plaintext is written, and every staging byte
 * (key, AD, input, output) is zeroed before the call returns, also on error
 * paths.  h_buf holds len plaintext bytes and has room for len+16 (encrypt),
 * or holds ct_len = len+16 bytes (decrypt, plaintext written to
 * h_buf[0..len) on success, h_buf untouched and NOISE_GPU_E_MAC returned on
 * failure).  An all-zero key returns NOISE_GPU_E_ARG (rekey excepted). */
int noise_gpu_encrypt_host(const uint8_t h_key[32], uint64_t nonce,
                           const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                           size_t len);
int noise_gpu_decrypt_host(const uint8_t h_key[32], uint64_t nonce,
                           const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                           size_t ct_len);
int noise_gpu_rekey_host(uint8_t h_key[32]);

/* Resident latency mode (opt-in) for the single-record entry points above,
 * for the calling thread on its current device.  on = 1: instead of one
 * kernel launch per record, ONE workgroup stays on the GPU and serves the
 * thread's records of up to 4032 bytes (<= 8192 bytes of AD):
 *   - the host writes each request into a request image in fine-grained
 *     device memory through the PCIe BAR: 16-byte chunks {seq, 12 bytes}
 *     carrying the key, nonce, lengths and -- for a staged image of up to
 *     1488 bytes -- the AD / record themselves, so the poll that finds the
 *     request has its data (larger ones follow by DMA);
 *   - output, status and the done word come back through the host-mapped
 *     staging image as in the launch path;
 *   - after answering (key, n) the workgroup precomputes (key, n + 1): its
 *     keystream and the Poly1305 powers r..r^192, two such slots (a session's
 *     two directions), so consecutive records of a CipherState are answered
 *     with one product per 16-byte block.
 * Records above 4032 bytes take a kernel launch on a second stream.  The
 * workgroup leaves on its own after idle_us microseconds without a request
 * (0 = the default, 20000; at most 10 s), is relaunched by the next request,
 * and is stopped by on = 0 (which also frees the request image),
 * noise_gpu_thread_release, thread exit and library unload; on the way out it
 * zeroes its LDS (speculated keystream, key copies).  While it runs it holds
 * one CU and ~105 KB of its LDS.
 *
 * Requests.  Each 16-byte chunk is written with ONE aligned 16-byte store
 * through the BAR (write-combined), after an sfence that orders it behind
 * the staged bytes.  The engine does not assume such a store lands whole:
 * chunk 3 carries a check word, a position-weighted sum of every payload word
 * of the header and inline chunks, and the workgroup takes a request only
 * when every chunk carries the new sequence number AND the words sum to the
 * check word -- a chunk seen half-landed (new sequence number, stale
 * payload) is polled again.  After ~4096 empty polls the polling wave backs
 * off (s_sleep between polls).
 *
 * Other work on the device.  The workgroup runs on a non-blocking stream of
 * the highest priority, whose hardware queue normal-priority streams never
 * share (the runtime maps streams onto a few hardware queues per priority, in
 * order: a stream sharing the instance's queue would wait until it idles
 * out).  A process that creates more high-priority streams of its own than
 * the runtime has queues (GPU_MAX_HW_QUEUES, default 4) may share it.  Device
 * memory the engine frees while running (records scratch that grows, staging,
 * a Pipeline's key table) is freed stream-ordered, so batch calls and
 * Pipelines on other threads never wait for the instance.  What still waits
 * for it to idle out (or for on = 0): hipDeviceSynchronize, hipFree and
 * hipHostFree (which on ROCm wait for every stream of the device) -- in the
 * engine: noise_gpu_ctx_destroy, noise_gpu_thread_release / thread exit of
 * ANOTHER thread, noise_gpu_hs_destroy, and a Pipeline's destructor.
 *
 * Stopping.  on = 0 sets the stop word and waits -- at most 10 s -- for the
 * workgroup's alive word before it synchronises the stream; an instance that
 * does not leave in that time makes the call fail with NOISE_GPU_E_HIP and
 * the context unusable (every later call on it fails; nothing it reads is
 * freed).  A request it does not answer within 10 s fails the same way.
 * Results, hygiene (the request image is zeroed, but for four sequence words,
 * before the done word) and error behaviour are those of the launch path.
 * NOISE_GPU_RESIDENT_REQ=host puts the request image in host-mapped memory
 * instead (polled over PCIe).  Records with more than 8192 bytes of AD or more
 * than 65535 bytes take the staged path either way. */
int noise_gpu_set_resident(int on, uint32_t idle_us);

/* Descriptor batch between HOST buffers (synchronous): the key table
 * (nkeys x 32 B), descriptors, h_in[0..in_bytes) and h_ad[0..ad_bytes) are
 * staged to the device, the records kernel runs, h_out[0..out_bytes) (and
 * h_status[nrec] for decrypt) are copied back.  Used by
 * CipherState::encrypt_batch / decrypt_batch.  Every descriptor range is
 * bounds-checked against its buffer on the host (overflow-safe), and the
 * device staging and the records scratch are zeroed before the call
 * returns. */
int noise_gpu_encrypt_records_host(const uint8_t *h_keys, uint32_t nkeys,
                                   const noise_gpu_record *h_recs,
                                   uint64_t nrec, const uint8_t *h_in,
                                   uint64_t in_bytes, uint8_t *h_out,
                                   uint64_t out_bytes, const uint8_t *h_ad,
                                   uint64_t ad_bytes);
int noise_gpu_decrypt_records_host(const uint8_t *h_keys, uint32_t nkeys,
                                   const noise_gpu_record *h_recs,
                                   uint64_t nrec, const uint8_t *h_in,
                                   uint64_t in_bytes, uint8_t *h_out,
                                   uint64_t out_bytes, const uint8_t *h_ad,
                                   uint64_t ad_bytes, uint8_t *h_status);

/* Uniform batch between HOST buffers: pinned-staged, chunked and
 * double-buffered (H2D copy || kernel || D2H copy on separate streams).
 * Encrypt: h_in records of len bytes (stride in_stride) -> h_out records of
 * len+16 (stride out_stride).  Decrypt: the reverse, with h_status[nrec].
 * *seconds receives the wall time of the whole call, from entry to return.
 * Streams, events and device buffers live in a context per (calling thread,
 * current device) that persists across calls (created on the thread's first
 * call on that device; a thread serving several GPUs keeps one per device);
 * their contents are zeroed at the end of every call.  The single-record
 * and descriptor host entry points above keep their staging the same way.
 * Footprint of that per-(thread, device) state: the uniform pipeline holds
 * 3 x 34 MiB of device memory and 3 streams; the descriptor path a device
 * staging buffer sized by the largest call plus its records scratch (about
 * 2 KiB per record of that call) and a companion stream; the single-record
 * path a pinned buffer.  It lives until the thread exits or calls
 * noise_gpu_thread_release() -- thread-pool servers should call that, or
 * use an explicit noise_gpu_ctx (below), whose destroy frees the same.
 * len is at most NOISE_GPU_UNIFORM_HOST_MAX_LEN (NOISE_GPU_E_ARG above it;
 * a Noise record is at most 65519 bytes). */
#define NOISE_GPU_UNIFORM_HOST_MAX_LEN (8u << 20)
int noise_gpu_encrypt_uniform_host(const uint8_t h_key[32], uint64_t nonce0,
                                   const uint8_t *h_in, uint64_t in_stride,
                                   uint8_t *h_out, uint64_t out_stride,
                                   uint32_t len, uint64_t nrec,
                                   double *seconds);
int noise_gpu_decrypt_uniform_host(const uint8_t h_key[32], uint64_t nonce0,
                                   const uint8_t *h_in, uint64_t in_stride,
                                   uint8_t *h_out, uint64_t out_stride,
                                   uint32_t len, uint8_t *h_status,
                                   uint64_t nrec, double *seconds);

/* Wipe and free every per-(calling thread, device) context the host-buffer
 * entry points created for this thread (staging, records scratch and its
 * companion stream, the latency-path buffer, the uniform pipeline), on all
 * devices.  The next call re-creates what it needs.  Synchronises the
 * thread's streams. */
int noise_gpu_thread_release(void);

/* ---- explicit device contexts --------------------------------------------
 * SURVEY 8(b) proposed noise_gpu_ctx_create(int device, ...).  The device-
 * resident entry points above need no context (a stream names the device's
 * work; the records scratch is kept per (device, stream)).  The host-buffer
 * entry points otherwise keep their staging per (calling thread, current
 * device); a noise_gpu_ctx instead owns that state for one device, so a
 * server can bind one context per GPU (or per connection thread) without
 * relying on hipSetDevice state.  Each noise_gpu_ctx_* call makes the
 * context's device current for its duration and restores the caller's
 * device afterwards; it behaves exactly like the context-free function of
 * the same name.  A context is not thread-safe: one thread at a time (like
 * a CipherState).  destroy wipes and frees everything the context staged,
 * including the descriptor path's records scratch and companion stream. */
typedef struct noise_gpu_ctx noise_gpu_ctx;
/* device: HIP device index (must be gfx950, else NOISE_GPU_E_NODEV) */
int noise_gpu_ctx_create(int device, noise_gpu_ctx **out);
int noise_gpu_ctx_destroy(noise_gpu_ctx *ctx);
int noise_gpu_ctx_device(const noise_gpu_ctx *ctx, int *device);
/* noise_gpu_set_resident for the context's single-record path; destroy
 * stops its resident workgroup. */
int noise_gpu_ctx_set_resident(noise_gpu_ctx *ctx, int on, uint32_t idle_us);
int noise_gpu_ctx_encrypt_host(noise_gpu_ctx *ctx, const uint8_t h_key[32], uint64_t nonce,
                               const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf, size_t len);
int noise_gpu_ctx_decrypt_host(noise_gpu_ctx *ctx, const uint8_t h_key[32], uint64_t nonce,
                               const uint8_t *h_ad, size_t ad_len, uint8_t *h_buf,
                               size_t ct_len);
int noise_gpu_ctx_rekey_host(noise_gpu_ctx *ctx, uint8_t h_key[32]);
int noise_gpu_ctx_encrypt_records_host(noise_gpu_ctx *ctx, const uint8_t *h_keys, uint32_t nkeys,
                                       const noise_gpu_record *h_recs, uint64_t nrec,
                                       const uint8_t *h_in, uint64_t in_bytes, uint8_t *h_out,
                                       uint64_t out_bytes, const uint8_t *h_ad,
                                       uint64_t ad_bytes);
int noise_gpu_ctx_decrypt_records_host(noise_gpu_ctx *ctx, const uint8_t *h_keys, uint32_t nkeys,
                                       const noise_gpu_record *h_recs, uint64_t nrec,
                                       const uint8_t *h_in, uint64_t in_bytes, uint8_t *h_out,
                                       uint64_t out_bytes, const uint8_t *h_ad,
                                       uint64_t ad_bytes, uint8_t *h_status);
int noise_gpu_ctx_encrypt_uniform_host(noise_gpu_ctx *ctx, const uint8_t h_key[32],
                                       uint64_t nonce0, const uint8_t *h_in, uint64_t in_stride,
                                       uint8_t *h_out, uint64_t out_stride, uint32_t len,
                                       uint64_t nrec, double *seconds);
int noise_gpu_ctx_decrypt_uniform_host(noise_gpu_ctx *ctx, const uint8_t h_key[32],
                                       uint64_t nonce0, const uint8_t *h_in, uint64_t in_stride,
                                       uint8_t *h_out, uint64_t out_stride, uint32_t len,
                                       uint8_t *h_status, uint64_t nrec, double *seconds);

/* ---- synthetic data (bench / tests) ------------------------------------
 * Fill d_dst[0..nbytes) with the splitmix64 stream: byte j = byte (j & 7)
 * of mix64(seed + ((offset+j)/8 + 1) * 0x9e3779b97f4a7c15), offset-relative
 * so shards of one logical buffer can be generated independently. */
int noise_gpu_fill_synthetic(uint8_t *d_dst, uint64_t offset, uint64_t nbytes,
                             uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NOISE_GPU_H */
