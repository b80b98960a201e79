// handshake.cpp -- SymmetricState / HandshakeState of the Noise Protocol
// Framework (rev34 §5.2-5.3, §7, §9) over BLAKE2b, X25519 and the GPU-backed
// CipherState.  Reference surface: noise.h:117-173; reference implementation
// noise.cpp:441-1100 (see handshake.hpp for where this one deliberately
// differs).
#include "noise_amd/handshake.hpp"

#include <cstring>
#include <stdexcept>

namespace noise {

namespace {
using crypto::Hash;
using crypto::kHashLen;
}  // namespace

KeyPair keypair_from_private(const std::array<std::uint8_t, 32> &sk) {
  KeyPair kp;
  kp.sk = sk;
  kp.pk = crypto::x25519_base(sk);
  return kp;
}

KeyPair generate_keypair() {
  std::array<std::uint8_t, 32> sk;
  crypto::random_bytes(sk.data(), sk.size());
  KeyPair kp = keypair_from_private(sk);
  crypto::wipe(sk.data(), sk.size());
  return kp;
}

// ---- SymmetricState (rev34 §5.2) ------------------------------------------
SymmetricState::~SymmetricState() {
  crypto::wipe(ck.data(), ck.size());
  crypto::wipe(h.data(), h.size());
}

void SymmetricState::initialize_symmetric(const std::vector<std::uint8_t> &protocol_name) {
  if (protocol_name.size() <= kHashLen) {
    h.fill(0);
    std::memcpy(h.data(), protocol_name.data(), protocol_name.size());
  } else {
    h = crypto::blake2b(protocol_name.data(), protocol_name.size());
  }
  ck = h;
  cs.initialize_key(std::array<std::uint8_t, 32>{});  // InitializeKey(empty)
}

void SymmetricState::mix_key(const std::uint8_t *ikm, std::size_t len) {
  Hash tk;
  crypto::hkdf(ck, ikm, len, &ck, &tk);
  std::array<std::uint8_t, 32> k;
  std::memcpy(k.data(), tk.data(), 32);  // HASHLEN 64: truncate to 32
  cs.initialize_key(k);
  crypto::wipe(tk.data(), tk.size());
  crypto::wipe(k.data(), k.size());
}

void SymmetricState::mix_hash(const std::uint8_t *data, std::size_t len) {
  crypto::Blake2b b;
  b.update(h.data(), h.size());
  if (len) b.update(data, len);
  b.final(h.data());
}

void SymmetricState::mix_key_and_hash(const std::uint8_t *ikm, std::size_t len) {
  Hash th, tk;
  crypto::hkdf(ck, ikm, len, &ck, &th, &tk);
  mix_hash(th.data(), th.size());
  std::array<std::uint8_t, 32> k;
  std::memcpy(k.data(), tk.data(), 32);
  cs.initialize_key(k);
  crypto::wipe(th.data(), th.size());
  crypto::wipe(tk.data(), tk.size());
  crypto::wipe(k.data(), k.size());
}

void SymmetricState::encrypt_and_hash(std::vector<std::uint8_t> &plaintext) {
  std::vector<std::uint8_t> ad(h.begin(), h.end());
  cs.encrypt_with_ad(ad, plaintext);  // no-op without a key (HasKey false)
  mix_hash(plaintext.data(), plaintext.size());
}

void SymmetricState::decrypt_and_hash(std::vector<std::uint8_t> &ciphertext) {
  const std::vector<std::uint8_t> ct(ciphertext);
  std::vector<std::uint8_t> ad(h.begin(), h.end());
  cs.decrypt_with_ad(ad, ciphertext);
  mix_hash(ct.data(), ct.size());
}

std::tuple<CipherState, CipherState> SymmetricState::split() {
  Hash t1, t2;
  crypto::hkdf(ck, nullptr, 0, &t1, &t2);
  std::array<std::uint8_t, 32> k1, k2;
  std::memcpy(k1.data(), t1.data(), 32);
  std::memcpy(k2.data(), t2.data(), 32);
  CipherState c1, c2;
  c1.initialize_key(k1);
  c2.initialize_key(k2);
  crypto::wipe(t1.data(), t1.size());
  crypto::wipe(t2.data(), t2.size());
  crypto::wipe(k1.data(), k1.size());
  crypto::wipe(k2.data(), k2.size());
  return {c1, c2};
}

// ---- HandshakeState (rev34 §5.3) ------------------------------------------
HandshakeState::~HandshakeState() {
  crypto::wipe(ssk.data(), ssk.size());
  crypto::wipe(esk.data(), esk.size());
  for (auto &p : psks) crypto::wipe(p.data(), p.size());
}

void HandshakeState::initialize(const HandshakeStateConfiguration &config) {
  initialize_named(pattern_name(config.pattern), config);
}


void HandshakeState::initialize_named(std::string_view pattern,
                                      const HandshakeStateConfiguration &config) {
  const detail::PatternProgram prog = detail::parse_pattern(pattern);
  initiator_pre_message_pattern = prog.pre_i;
  responder_pre_message_pattern = prog.pre_r;
  message_patterns.assign(prog.msgs.begin(), prog.msgs.end());
  psk_mode = prog.psk_mode;
  if (config.psks.size() != prog.npsk) throw std::invalid_argument("psk count does not match the pattern");
  psks.assign(config.psks.begin(), config.psks.end());
  for (const auto &p : psks)
    if (p.size() != 32) throw std::invalid_argument("psk must be 32 bytes");

  initiator = config.initiator;
  my_turn = initiator;
  completed = false;
  result.reset();
  has_s = config.s.has_value();
  has_e = config.e.has_value();
  has_rs = config.rs.has_value();
  has_re = config.re.has_value();
  if (has_s) { ssk = config.s->sk; spk = config.s->pk; }
  if (has_e) { esk = config.e->sk; epk = config.e->pk; }
  if (has_rs) rspk = *config.rs;
  if (has_re) repk = *config.re;

  const std::string name = "Noise_" + std::string(pattern) + "_25519_ChaChaPoly_BLAKE2b";
  ss.initialize_symmetric(std::vector<std::uint8_t>(name.begin(), name.end()));
  ss.mix_hash(config.prologue);
  // pre-messages: the initiator's keys first, then the responder's (§5.3)
  auto pre = [&](const std::vector<PatternToken> &toks, bool initiators) {
    const bool mine = initiators == initiator;
    for (PatternToken t : toks) {
      if (t == PatternToken::S) {
        if (!(mine ? has_s : has_rs)) throw std::invalid_argument("pre-message static key missing");
        ss.mix_hash(mine ? spk : rspk);
      } else if (t == PatternToken::E) {
        if (!(mine ? has_e : has_re)) throw std::invalid_argument("pre-message ephemeral key missing");
        ss.mix_hash(mine ? epk : repk);
        if (psk_mode) ss.mix_key(mine ? epk : repk);
      } else {
        throw std::logic_error("bad pre-message token");
      }
    }
  };
  pre(initiator_pre_message_pattern, true);
  pre(responder_pre_message_pattern, false);
}

void HandshakeState::dh_mix(PatternToken t) {
  const std::array<std::uint8_t, 32> *sk = nullptr, *pk = nullptr;
  bool ok = false;
  switch (t) {
    case PatternToken::Ee:
      sk = &esk; pk = &repk; ok = has_e && has_re;
      break;
    case PatternToken::Ss:
      sk = &ssk; pk = &rspk; ok = has_s && has_rs;
      break;
    case PatternToken::Es:  // initiator: DH(e, rs); responder: DH(s, re)
      if (initiator) { sk = &esk; pk = &rspk; ok = has_e && has_rs; }
      else { sk = &ssk; pk = &repk; ok = has_s && has_re; }
      break;
    case PatternToken::Se:  // initiator: DH(s, re); responder: DH(e, rs)
      if (initiator) { sk = &ssk; pk = &repk; ok = has_s && has_re; }
      else { sk = &esk; pk = &rspk; ok = has_e && has_rs; }
      break;
    default:
      throw std::logic_error("not a DH token");
  }
  if (!ok) throw std::logic_error("DH with a missing key");
  std::array<std::uint8_t, 32> shared = crypto::x25519(*sk, *pk);
  ss.mix_key(shared);
  crypto::wipe(shared.data(), shared.size());
}

void HandshakeState::finish_if_done() {
  my_turn = !my_turn;
  if (message_patterns.empty()) {
    completed = true;
    result = ss.split();
  }
}

void HandshakeState::write_message(std::vector<std::uint8_t> &payload,
                                   std::vector<std::uint8_t> &message_buffer) {
  if (completed) throw std::runtime_error("Handshake has already been completed!");  // noise.cpp:879-881
  if (!my_turn)  // noise.cpp:882-885
    throw std::runtime_error("Expected a read message call, but write message was called instead!");
  if (payload.size() > 65535) throw std::length_error("payload exceeds 65535 bytes");
  const std::size_t start = message_buffer.size();
  for (PatternToken t : message_patterns.front()) {
    switch (t) {
      case PatternToken::E: {
        if (!has_e) {  // spec: GENERATE_KEYPAIR unless pre-set (test vectors)
          const KeyPair kp = generate_keypair();
          esk = kp.sk;
          epk = kp.pk;
          has_e = true;
        }
        message_buffer.insert(message_buffer.end(), epk.begin(), epk.end());
        ss.mix_hash(epk);
        if (psk_mode) ss.mix_key(epk);
        break;
      }
      case PatternToken::S: {
        if (!has_s) throw std::logic_error("static key missing");
        std::vector<std::uint8_t> tmp(spk.begin(), spk.end());
        ss.encrypt_and_hash(tmp);
        message_buffer.insert(message_buffer.end(), tmp.begin(), tmp.end());
        break;
      }
      case PatternToken::Psk: {
        if (psks.empty()) throw std::logic_error("psk missing");
        ss.mix_key_and_hash(psks.front());
        crypto::wipe(psks.front().data(), psks.front().size());
        psks.pop_front();
        break;
      }
      default:
        dh_mix(t);
    }
  }
  std::vector<std::uint8_t> body(payload);
  ss.encrypt_and_hash(body);
  message_buffer.insert(message_buffer.end(), body.begin(), body.end());
  if (message_buffer.size() - start > 65535) throw std::length_error("message exceeds 65535 bytes");
  message_patterns.pop_front();
  finish_if_done();
}

void HandshakeState::write_message(std::vector<std::uint8_t> &message_buffer) {
  std::vector<std::uint8_t> empty;
  write_message(empty, message_buffer);
}

void HandshakeState::read_message(std::vector<std::uint8_t> &message,
                                  std::vector<std::uint8_t> &payload_buffer) {
  if (completed) throw std::runtime_error("Handshake has already been completed!");  // noise.cpp:975-977
  if (my_turn)  // noise.cpp:978-981
    throw std::runtime_error("Expected a write message call, but read message was called instead!");
  if (message.size() > 65535) throw std::length_error("message exceeds 65535 bytes");
  std::size_t off = 0;
  auto take = [&](std::size_t n) {
    if (message.size() - off < n) throw std::invalid_argument("handshake message too short");
    std::vector<std::uint8_t> v(message.begin() + off, message.begin() + off + n);
    off += n;
    return v;
  };
  for (PatternToken t : message_patterns.front()) {
    switch (t) {
      case PatternToken::E: {
        const std::vector<std::uint8_t> v = take(32);
        std::memcpy(repk.data(), v.data(), 32);
        has_re = true;
        ss.mix_hash(repk);
        if (psk_mode) ss.mix_key(repk);
        break;
      }
      case PatternToken::S: {
        std::vector<std::uint8_t> v = take(ss.cs_has_key() ? 32 + 16 : 32);
        ss.decrypt_and_hash(v);  // throws invalid_argument on a bad tag
        std::memcpy(rspk.data(), v.data(), 32);
        has_rs = true;
        break;
      }
      case PatternToken::Psk: {
        if (psks.empty()) throw std::logic_error("psk missing");
        ss.mix_key_and_hash(psks.front());
        crypto::wipe(psks.front().data(), psks.front().size());
        psks.pop_front();
        break;
      }
      default:
        dh_mix(t);
    }
  }
  std::vector<std::uint8_t> body(message.begin() + off, message.end());
  ss.decrypt_and_hash(body);
  payload_buffer.insert(payload_buffer.end(), body.begin(), body.end());
  message_patterns.pop_front();
  finish_if_done();
}

std::tuple<CipherState, CipherState> HandshakeState::finalize() {
  if (!completed || !result) throw std::logic_error("handshake not finished");
  return *result;
}

}  // namespace noise
