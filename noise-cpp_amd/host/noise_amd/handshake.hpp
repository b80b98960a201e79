// noise_amd/handshake.hpp -- spec-correct Noise handshake on the host whose
// split() hands out GPU-backed noise::CipherState pairs.
//
// Surface of the reference's noise.h:19-97, 117-173 (PatternToken,
// HandshakePattern with the same 59 names, KeyPair, generate_keypair,
// HandshakeStateConfiguration, SymmetricState, HandshakeState with
// initialize / write_message / read_message / get_* / finalize), suite fixed
// to Noise_*_25519_ChaChaPoly_BLAKE2b as in the reference (noise.cpp:547-548).
// The transport CipherStates are noise_amd/cipher_state.hpp (every AEAD byte
// on the MI355X); the handshake's own EncryptAndHash / DecryptAndHash go
// through the same CipherState.
//
// Deliberate differences from the reference implementation (noise.cpp) --
// each one a reference bug that breaks interoperability:
//  * encryption follows HasKey() of the spec (the reference's inverted
//    has_key encrypts handshake payloads under the all-zero key and sends
//    transport records in the clear: Q1);
//  * a pre-set ephemeral key (HandshakeStateConfiguration::e) is used, as the
//    spec allows for test vectors (the reference throws, noise.cpp:896-900);
//  * psk patterns keep the caller's psks (the reference copies them into an
//    empty vector and crashes, noise.cpp:588: Q6);
//  * the responder's pre-message pattern is processed (the reference walks
//    the initiator's twice, noise.cpp:819-871: Q7).
// Besides the enum, initialize_named() accepts any pattern name of the
// fundamental/one-way/deferred table with psk modifiers (e.g.
// "XXpsk0+psk2"), which the test vectors use.
#pragma once
#include <array>
#include <cstdint>
#include <deque>
#include <optional>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

#include "noise_amd/cipher_state.hpp"
#include "noise_amd/crypto.hpp"

namespace noise {

enum class PatternToken : std::uint8_t { E, S, Ee, Es, Se, Ss, Psk };

enum class HandshakePattern : std::uint8_t {
  IK, IN, IX, K, KK, KN, KX, N, NK, NN, NX, XK, XN, XX,
  NK1, NX1, X, X1K, XK1, X1K1, X1N, X1X, XX1, X1X1, K1N, K1K, KK1, K1K1, K1X,
  KX1, K1X1, I1N, I1K, IK1, I1K1, I1X, IX1, I1X1,
  Npsk0, Kpsk0, Xpsk1, NNpsk0, NNpsk2, NKpsk0, NKpsk2, NXpsk2, XNpsk3, XKpsk3,
  XXpsk3, KNpsk0, KNpsk2, KKpsk0, KKpsk2, KXpsk2, INpsk1, INpsk2, IKpsk1,
  IKpsk2, IXpsk2,
};

// pattern name as it appears in the protocol name ("XXpsk3")
std::string_view pattern_name(HandshakePattern p);

namespace detail {
// A pattern name with psk modifiers ("XXpsk0+psk2") parsed into its
// pre-messages and per-message token lists (rev34 §7, §9; the reference's
// table is noise.cpp:594-818).  Shared by HandshakeState and the batched GPU
// handshake (noise_gpu_hs_*).  Throws std::logic_error for unknown names.
struct PatternProgram {
  std::vector<PatternToken> pre_i, pre_r;
  std::vector<std::vector<PatternToken>> msgs;
  std::size_t npsk = 0;
  bool psk_mode = false;
  bool one_way = false;  // N, K, X and their psk variants: initiator writes all
};
PatternProgram parse_pattern(std::string_view name);
}  // namespace detail

struct KeyPair {
  std::array<std::uint8_t, 32> sk;
  std::array<std::uint8_t, 32> pk;
};

KeyPair generate_keypair();
// the key pair of a given private key (pk = X25519(sk, 9))
KeyPair keypair_from_private(const std::array<std::uint8_t, 32> &sk);

struct HandshakeStateConfiguration {
  HandshakePattern pattern;
  bool initiator;
  std::vector<std::uint8_t> prologue;
  std::optional<KeyPair> s, e;
  std::optional<std::array<std::uint8_t, 32>> rs, re;
  std::vector<std::vector<std::uint8_t>> psks;
};

class SymmetricState {
 private:
  CipherState cs;
  std::array<std::uint8_t, 64> ck;
  std::array<std::uint8_t, 64> h;

 public:
  SymmetricState() = default;
  ~SymmetricState();
  void initialize_symmetric(const std::vector<std::uint8_t> &protocol_name);
  void mix_key(const std::uint8_t *ikm, std::size_t len);
  void mix_hash(const std::uint8_t *data, std::size_t len);
  void mix_key_and_hash(const std::uint8_t *ikm, std::size_t len);
  template <STLContainer T> void mix_key(T &ikm) { mix_key(bytes(ikm), ikm.size()); }
  template <STLContainer T> void mix_hash(const T &data) {
    mix_hash(reinterpret_cast<const std::uint8_t *>(data.data()), data.size());
  }
  template <STLContainer T> void mix_key_and_hash(T &ikm) {
    mix_key_and_hash(bytes(ikm), ikm.size());
  }
  [[nodiscard]] std::array<std::uint8_t, 64> get_handshake_hash() const { return h; }
  // in place: plaintext -> ciphertext (grows by 16 once a key is set)
  void encrypt_and_hash(std::vector<std::uint8_t> &plaintext);
  // in place: ciphertext -> plaintext; throws invalid_argument("Invalid MAC")
  void decrypt_and_hash(std::vector<std::uint8_t> &ciphertext);
  [[nodiscard]] std::tuple<CipherState, CipherState> split();
  [[nodiscard]] bool cs_has_key() const { return cs.has_key(); }

 private:
  template <class T> static const std::uint8_t *bytes(const T &c) {
    return reinterpret_cast<const std::uint8_t *>(c.data());
  }
};

class HandshakeState {
 private:
  SymmetricState ss;
  std::array<std::uint8_t, 32> spk{}, ssk{}, epk{}, esk{}, rspk{}, repk{};
  bool has_s = false, has_e = false, has_rs = false, has_re = false;
  bool initiator = false, my_turn = false, completed = false, psk_mode = false;
  std::deque<std::vector<PatternToken>> message_patterns;
  std::vector<PatternToken> initiator_pre_message_pattern, responder_pre_message_pattern;
  std::deque<std::vector<std::uint8_t>> psks;
  std::optional<std::tuple<CipherState, CipherState>> result;

  void dh_mix(PatternToken t);
  void finish_if_done();

 public:
  HandshakeState() = default;
  ~HandshakeState();
  void initialize(const HandshakeStateConfiguration &config);
  // pattern by name (superset of the enum: any psk modifier list)
  void initialize_named(std::string_view pattern, const HandshakeStateConfiguration &config);
  // WriteMessage(payload, message_buffer): appends the handshake message
  void write_message(std::vector<std::uint8_t> &payload,
                     std::vector<std::uint8_t> &message_buffer);
  void write_message(std::vector<std::uint8_t> &message_buffer);
  // ReadMessage(message, payload_buffer): appends the decrypted payload
  void read_message(std::vector<std::uint8_t> &message,
                    std::vector<std::uint8_t> &payload_buffer);
  [[nodiscard]] std::array<std::uint8_t, 64> get_handshake_hash() { return ss.get_handshake_hash(); }
  [[nodiscard]] std::array<std::uint8_t, 32> get_local_static_public_key() { return spk; }
  [[nodiscard]] std::array<std::uint8_t, 32> get_local_ephemeral_public_key() { return epk; }
  [[nodiscard]] std::array<std::uint8_t, 32> get_remote_ephemeral_public_key() { return repk; }
  [[nodiscard]] std::array<std::uint8_t, 32> get_remote_static_public_key() { return rspk; }
  [[nodiscard]] bool is_initiator() { return initiator; }
  [[nodiscard]] bool is_handshake_finished() { return completed; }
  [[nodiscard]] bool is_my_turn() { return my_turn; }
  // (c1, c2) of Split(): c1 encrypts initiator -> responder
  [[nodiscard]] std::tuple<CipherState, CipherState> finalize();
};

}  // namespace noise
