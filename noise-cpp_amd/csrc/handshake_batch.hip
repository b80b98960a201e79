// handshake_batch.hip -- the noise_gpu_hs_* C ABI (include/noise_gpu.h): the
// host side of batched handshakes.  It walks the pattern's token program
// (noise::detail::parse_pattern, shared with the host HandshakeState) and
// launches one kernel of handshake_kernels.hip per token over all sessions;
// everything that is the same for every session -- HasKey(), the handshake
// nonce n, message cursors and lengths of the fixed parts -- is tracked here,
// exactly as noise::HandshakeState tracks it for one session
// (host/handshake.cpp, noise.cpp:545-1100).  No cryptography runs on the host
// except the protocol-name hash (one BLAKE2b per batch) and the 32-byte DRBG
// seed from getrandom per generated ephemeral.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "launchers.hpp"
#include "noise_amd/crypto.hpp"
#include "noise_amd/handshake.hpp"

using noise::PatternToken;
using namespace noise_amd;

struct noise_gpu_hs {
  noise::detail::PatternProgram prog;
  std::string name;
  bool initiator = false;
  uint64_t n = 0;
  HsSession *S = nullptr;
  uint8_t *psks = nullptr;
  bool has[6] = {};       // HsKey slots present (s/spk, e/epk, rs, re)
  bool psks_set = false;
  bool started = false;
  bool has_k = false;     // HasKey() of the handshake CipherState
  uint64_t nonce = 0;     // its n
  size_t msg = 0;         // next message index
  size_t psk_next = 0;
  uint32_t drbg_ctr = 0;
};

namespace {

#define HS_TRY(expr)                                          \
  do {                                                        \
    hipError_t e_ = (expr);                                   \
    if (e_ != hipSuccess) return api_hip_fail(e_, #expr);     \
  } while (0)

bool my_turn(const noise_gpu_hs *hs) {
  if (hs->prog.one_way) return hs->initiator;
  return ((hs->msg % 2) == 0) == hs->initiator;
}

// Fixed bytes of the next message (tokens + payload tag), from the current
// HasKey() -- the same walk write/read make, without side effects.
uint32_t overhead(const noise_gpu_hs *hs) {
  if (hs->msg >= hs->prog.msgs.size()) return 0;
  bool k = hs->has_k;
  uint32_t bytes = 0;
  for (PatternToken t : hs->prog.msgs[hs->msg]) {
    switch (t) {
      case PatternToken::E:
        bytes += 32;
        if (hs->prog.psk_mode) k = true;
        break;
      case PatternToken::S:
        bytes += k ? 48 : 32;
        break;
      default:  // DH tokens and psk all MixKey
        k = true;
    }
  }
  return bytes + (k ? 16 : 0);
}

// (private, public) slots of a DH token for this role (rev34 §5.3 / host dh_mix)
bool dh_slots(const noise_gpu_hs *hs, PatternToken t, int &sk, int &pk) {
  switch (t) {
    case PatternToken::Ee: sk = kHsEsk; pk = kHsRe; break;
    case PatternToken::Ss: sk = kHsSsk; pk = kHsRs; break;
    case PatternToken::Es:
      if (hs->initiator) { sk = kHsEsk; pk = kHsRs; }
      else { sk = kHsSsk; pk = kHsRe; }
      break;
    case PatternToken::Se:
      if (hs->initiator) { sk = kHsSsk; pk = kHsRe; }
      else { sk = kHsEsk; pk = kHsRs; }
      break;
    default:
      return false;
  }
  // private slots are present when their public half is
  const int need_sk = sk == kHsEsk ? kHsEpk : kHsSpk;
  return hs->has[need_sk] && hs->has[pk];
}

HsSpan span_of(const noise_gpu_span *s) {
  HsSpan o{};
  if (!s) return o;
  o.base = s->base;
  o.off = s->off;
  o.stride = s->stride;
  o.len = s->len;
  o.len_u = s->len_all;
  return o;
}

HsWords8 drbg_seed() {
  HsWords8 w;
  noise::crypto::random_bytes(reinterpret_cast<uint8_t *>(w.w), sizeof(w.w));
  return w;
}

void wipe_words(HsWords8 &w) { noise::crypto::wipe(w.w, sizeof(w.w)); }

}  // namespace

extern "C" {

int noise_gpu_hs_create(const char *pattern, int initiator, uint64_t n, noise_gpu_hs **out) {
  if (!pattern || !out) return api_arg_fail("null pattern / output");
  *out = nullptr;
  if (n == 0) return api_arg_fail("a handshake batch needs n >= 1 sessions");
  noise_gpu_hs *hs = new (std::nothrow) noise_gpu_hs();
  if (!hs) return api_arg_fail("out of host memory");
  try {
    hs->prog = noise::detail::parse_pattern(pattern);
  } catch (const std::exception &e) {
    delete hs;
    return api_arg_fail(e.what());
  }
  const int rc = api_check_device();
  if (rc) {
    delete hs;
    return rc;
  }
  hs->name = pattern;
  hs->initiator = initiator != 0;
  hs->n = n;
  hipError_t e = hipMalloc(&hs->S, n * sizeof(HsSession));
  if (e == hipSuccess) e = hipMemset(hs->S, 0, n * sizeof(HsSession));
  if (e == hipSuccess && hs->prog.npsk) e = hipMalloc(&hs->psks, n * hs->prog.npsk * 32);
  if (e != hipSuccess) {
    if (hs->S) (void)hipFree(hs->S);
    delete hs;
    return api_hip_fail(e, "handshake batch allocation");
  }
  *out = hs;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_destroy(noise_gpu_hs *hs) {
  if (!hs) return NOISE_GPU_OK;
  int rc = NOISE_GPU_OK;
  if (hs->S) {
    if (launch_hs_wipe(hs->S, hs->n, nullptr) != hipSuccess) rc = NOISE_GPU_E_HIP;
    if (hipDeviceSynchronize() != hipSuccess) rc = NOISE_GPU_E_HIP;
    (void)hipFree(hs->S);
  }
  if (hs->psks) {
    (void)hipMemset(hs->psks, 0, hs->n * hs->prog.npsk * 32);
    (void)hipDeviceSynchronize();
    (void)hipFree(hs->psks);
  }
  delete hs;
  return rc;
}

int noise_gpu_hs_info_get(const noise_gpu_hs *hs, noise_gpu_hs_info *out) {
  if (!hs || !out) return api_arg_fail("null batch / output");
  out->message_index = (uint32_t)hs->msg;
  out->message_count = (uint32_t)hs->prog.msgs.size();
  out->finished = hs->msg >= hs->prog.msgs.size();
  out->my_turn = !out->finished && my_turn(hs);
  out->overhead = overhead(hs);
  out->psk_count = (uint32_t)hs->prog.npsk;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_set_key(noise_gpu_hs *hs, int which, const uint8_t *d_keys, uint64_t stride,
                         void *stream) {
  if (!hs || !d_keys) return api_arg_fail("null batch / keys");
  if (hs->started) return api_arg_fail("keys are set before noise_gpu_hs_start");
  const hipStream_t st = (hipStream_t)stream;
  int slot;
  bool derive;
  switch (which) {
    case NOISE_GPU_HS_S: slot = kHsSsk; derive = true; break;
    case NOISE_GPU_HS_E: slot = kHsEsk; derive = true; break;
    case NOISE_GPU_HS_RS: slot = kHsRs; derive = false; break;
    case NOISE_GPU_HS_RE: slot = kHsRe; derive = false; break;
    default: return api_arg_fail("unknown key slot");
  }
  HsWords8 none{};
  // stride 0: one key for every session -- install (and derive) it in row 0
  // only, then copy the row-0 slots to the others
  HS_TRY(launch_hs_set_key(hs->S, stride ? hs->n : 1, slot, d_keys, stride, none, 0, derive, st));
  if (!stride) HS_TRY(launch_hs_bcast_key(hs->S, hs->n, slot, derive ? 2 : 1, st));
  hs->has[slot] = true;
  if (derive) hs->has[slot + 1] = true;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_set_psks(noise_gpu_hs *hs, const uint8_t *d_psks, void *stream) {
  if (!hs || !d_psks) return api_arg_fail("null batch / psks");
  if (hs->started) return api_arg_fail("psks are set before noise_gpu_hs_start");
  if (!hs->prog.npsk) return api_arg_fail("the pattern has no psk modifier");
  HS_TRY(hipMemcpyAsync(hs->psks, d_psks, hs->n * hs->prog.npsk * 32, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  hs->psks_set = true;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_start(noise_gpu_hs *hs, const noise_gpu_span *prologue, void *stream) {
  if (!hs) return api_arg_fail("null batch");
  if (hs->started) return api_arg_fail("batch already started");
  if (hs->prog.npsk && !hs->psks_set) return api_arg_fail("psk pattern without psks");
  const hipStream_t st = (hipStream_t)stream;
  // InitializeSymmetric: h = protocol name padded, or its hash if > 64 bytes
  const std::string name = "Noise_" + hs->name + "_25519_ChaChaPoly_BLAKE2b";
  HsWords16 h0{};
  if (name.size() <= 64) {
    std::memcpy(h0.w, name.data(), name.size());
  } else {
    const noise::crypto::Hash d =
        noise::crypto::blake2b(reinterpret_cast<const uint8_t *>(name.data()), name.size());
    std::memcpy(h0.w, d.data(), 64);
  }
  HS_TRY(launch_hs_init(hs->S, hs->n, h0, span_of(prologue), st));
  // pre-messages: the initiator's keys first, then the responder's
  for (int side = 0; side < 2; ++side) {
    const bool mine = (side == 0) == hs->initiator;
    for (PatternToken t : side == 0 ? hs->prog.pre_i : hs->prog.pre_r) {
      int slot;
      if (t == PatternToken::S) slot = mine ? kHsSpk : kHsRs;
      else if (t == PatternToken::E) slot = mine ? kHsEpk : kHsRe;
      else return api_arg_fail("bad pre-message token");
      if (!hs->has[slot]) return api_arg_fail("pre-message key missing (noise_gpu_hs_set_key)");
      const bool key = t == PatternToken::E && hs->prog.psk_mode;
      HS_TRY(launch_hs_key_token(hs->S, hs->n, slot, 0, HsSpan{}, true, key, st));
      if (key) {
        hs->has_k = true;
        hs->nonce = 0;
      }
    }
  }
  hs->started = true;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_write_message(noise_gpu_hs *hs, const noise_gpu_span *payload,
                               const noise_gpu_span *msg, uint32_t *d_msg_len, void *stream) {
  if (!hs || !msg || !msg->base) return api_arg_fail("null batch / message span");
  if (!hs->started) return api_arg_fail("noise_gpu_hs_start first");
  if (hs->msg >= hs->prog.msgs.size()) return api_arg_fail("handshake already finished");
  if (!my_turn(hs)) return api_arg_fail("not this party's turn to write");
  const hipStream_t st = (hipStream_t)stream;
  const uint64_t n = hs->n;
  // the whole message (token bytes + payload + tag) must fit 65535 bytes, as
  // the host HandshakeState throws length_error (noise.cpp:886): uniform
  // lengths are refused here, per-session lengths fail their sessions with
  // BAD_LEN on the device before any byte is written
  const uint32_t need = overhead(hs);
  if (payload && !payload->len && (uint64_t)payload->len_all + need > 65535)
    return api_arg_fail("message (payload + overhead) exceeds 65535 bytes");
  if (payload && payload->len) HS_TRY(launch_hs_check_len(hs->S, n, payload->len, need, need, st));
  HsSpan m = span_of(msg);
  m.len = nullptr;
  for (PatternToken t : hs->prog.msgs[hs->msg]) {
    switch (t) {
      case PatternToken::E: {
        if (!hs->has[kHsEpk]) {  // GENERATE_KEYPAIR on the device DRBG
          HsWords8 seed = drbg_seed();
          const hipError_t e =
              launch_hs_set_key(hs->S, n, kHsEsk, nullptr, 0, seed, hs->drbg_ctr++, true, st);
          wipe_words(seed);
          HS_TRY(e);
          hs->has[kHsEsk] = hs->has[kHsEpk] = true;
        }
        HS_TRY(launch_hs_key_token(hs->S, n, kHsEpk, 1, m, true, hs->prog.psk_mode, st));
        m.add += 32;
        if (hs->prog.psk_mode) {
          hs->has_k = true;
          hs->nonce = 0;
        }
        break;
      }
      case PatternToken::S: {
        if (!hs->has[kHsSpk]) return api_arg_fail("static key missing");
        HS_TRY(launch_hs_encrypt_hash(hs->S, n, hs->has_k, hs->nonce, kHsSpk, HsSpan{}, m,
                                      nullptr, st));
        m.add += hs->has_k ? 48 : 32;
        if (hs->has_k) ++hs->nonce;
        break;
      }
      case PatternToken::Psk: {
        HS_TRY(launch_hs_psk(hs->S, n, hs->psks, (uint32_t)hs->prog.npsk,
                             (uint32_t)hs->psk_next++, st));
        hs->has_k = true;
        hs->nonce = 0;
        break;
      }
      default: {
        int sk, pk;
        if (!dh_slots(hs, t, sk, pk)) return api_arg_fail("DH with a missing key");
        HS_TRY(launch_hs_dh(hs->S, n, sk, pk, st));
        hs->has_k = true;
        hs->nonce = 0;
      }
    }
  }
  HsSpan p = span_of(payload);
  if (!payload) p.base = m.base;  // empty payloads: len 0, never dereferenced
  HS_TRY(launch_hs_encrypt_hash(hs->S, n, hs->has_k, hs->nonce, -1, p, m, d_msg_len, st));
  if (hs->has_k) ++hs->nonce;
  ++hs->msg;
  return NOISE_GPU_OK;
}

int noise_gpu_hs_read_message(noise_gpu_hs *hs, const noise_gpu_span *msg,
                              const noise_gpu_span *payload, uint32_t *d_payload_len,
                              uint8_t *d_status, void *stream) {
  if (!hs || !msg || !msg->base) return api_arg_fail("null batch / message span");
  if (!hs->started) return api_arg_fail("noise_gpu_hs_start first");
  if (hs->msg >= hs->prog.msgs.size()) return api_arg_fail("handshake already finished");
  if (my_turn(hs)) return api_arg_fail("not this party's turn to read");
  const hipStream_t st = (hipStream_t)stream;
  const uint64_t n = hs->n;
  const uint32_t need = overhead(hs);
  if (msg->len) {
    HS_TRY(launch_hs_check_len(hs->S, n, msg->len, need, 0, st));
  } else if (msg->len_all < need || msg->len_all > 65535) {
    return api_arg_fail("message length outside [overhead, 65535]");
  }
  if (!payload && msg->len) return api_arg_fail("per-session message lengths need a payload span");
  if (!payload && msg->len_all != need) return api_arg_fail("non-empty payloads need a payload span");
  HsSpan m = span_of(msg);
  for (PatternToken t : hs->prog.msgs[hs->msg]) {
    switch (t) {
      case PatternToken::E: {
        HS_TRY(launch_hs_key_token(hs->S, n, kHsRe, 2, m, true, hs->prog.psk_mode, st));
        hs->has[kHsRe] = true;
        m.add += 32;
        if (hs->prog.psk_mode) {
          hs->has_k = true;
          hs->nonce = 0;
        }
        break;
      }
      case PatternToken::S: {
        HsSpan c = m;
        c.len = nullptr;
        c.len_u = hs->has_k ? 48 : 32;
        HS_TRY(launch_hs_decrypt_hash(hs->S, n, hs->has_k, hs->nonce, c, kHsRs, HsSpan{}, nullptr,
                                      st));
        hs->has[kHsRs] = true;
        m.add += c.len_u;
        if (hs->has_k) ++hs->nonce;
        break;
      }
      case PatternToken::Psk: {
        HS_TRY(launch_hs_psk(hs->S, n, hs->psks, (uint32_t)hs->prog.npsk,
                             (uint32_t)hs->psk_next++, st));
        hs->has_k = true;
        hs->nonce = 0;
        break;
      }
      default: {
        int sk, pk;
        if (!dh_slots(hs, t, sk, pk)) return api_arg_fail("DH with a missing key");
        HS_TRY(launch_hs_dh(hs->S, n, sk, pk, st));
        hs->has_k = true;
        hs->nonce = 0;
      }
    }
  }
  // the payload ciphertext: the rest of the message
  HsSpan c = m;
  if (c.len) c.len_adj = -(int32_t)c.add;
  else c.len_u = msg->len_all - c.add;
  HsSpan p = span_of(payload);
  if (!payload) p.base = m.base;  // empty payloads: nothing is written
  HS_TRY(launch_hs_decrypt_hash(hs->S, n, hs->has_k, hs->nonce, c, -1, p, d_payload_len, st));
  if (hs->has_k) ++hs->nonce;
  ++hs->msg;
  if (d_status) HS_TRY(launch_hs_status(hs->S, n, d_status, st));
  return NOISE_GPU_OK;
}

int noise_gpu_hs_status(const noise_gpu_hs *hs, uint8_t *d_status, void *stream) {
  if (!hs || !d_status) return api_arg_fail("null batch / status");
  HS_TRY(launch_hs_status(hs->S, hs->n, d_status, (hipStream_t)stream));
  return NOISE_GPU_OK;
}

int noise_gpu_hs_split(noise_gpu_hs *hs, uint8_t *d_k1, uint8_t *d_k2, uint8_t *d_hash,
                       uint8_t *d_rs, void *stream) {
  if (!hs || !d_k1 || !d_k2) return api_arg_fail("null batch / key tables");
  if (hs->msg < hs->prog.msgs.size()) return api_arg_fail("handshake not finished");
  if (((reinterpret_cast<uintptr_t>(d_k1) | reinterpret_cast<uintptr_t>(d_k2) |
        reinterpret_cast<uintptr_t>(d_hash) | reinterpret_cast<uintptr_t>(d_rs)) & 15u) != 0)
    return api_arg_fail("split outputs must be 16-byte aligned");
  if (d_rs && !hs->has[kHsRs]) return api_arg_fail("no remote static key in this pattern");
  HS_TRY(launch_hs_split(hs->S, hs->n, d_k1, d_k2, d_hash, d_rs, (hipStream_t)stream));
  return NOISE_GPU_OK;
}

}  // extern "C"
