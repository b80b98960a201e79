// patterns.cpp -- the handshake pattern table of Noise rev34 §7.4-7.5 and
// §18 (deferred patterns) with psk modifiers (§9), parsed into token
// programs.  Shared by the host HandshakeState (handshake.cpp) and the batched
// GPU handshake (csrc/handshake_batch.hip); no cryptography and no device
// code, so it also links into the CPU emulation of the handshake kernels.
// The reference's table: noise.cpp:33-162 (names), 594-818 (tokens).
#include <stdexcept>
#include <string>

#include "noise_amd/handshake.hpp"

namespace noise {

namespace {
// ---- pattern table (Noise rev34 §7.4-7.5, §18 deferred patterns) ----------
// pre-messages and messages as token strings; messages alternate
// initiator -> responder -> initiator ...
struct PatternDef {
  const char *name, *pre_i, *pre_r, *msgs;
};
constexpr PatternDef kPatterns[] = {
    {"N", "", "s", "e,es"},
    {"K", "s", "s", "e,es,ss"},
    {"X", "", "s", "e,es,s,ss"},
    {"NN", "", "", "e|e,ee"},
    {"NK", "", "s", "e,es|e,ee"},
    {"NX", "", "", "e|e,ee,s,es"},
    {"XN", "", "", "e|e,ee|s,se"},
    {"XK", "", "s", "e,es|e,ee|s,se"},
    {"XX", "", "", "e|e,ee,s,es|s,se"},
    {"KN", "s", "", "e|e,ee,se"},
    {"KK", "s", "s", "e,es,ss|e,ee,se"},
    {"KX", "s", "", "e|e,ee,se,s,es"},
    {"IN", "", "", "e,s|e,ee,se"},
    {"IK", "", "s", "e,es,s,ss|e,ee,se"},
    {"IX", "", "", "e,s|e,ee,se,s,es"},
    {"NK1", "", "s", "e|e,ee,es"},
    {"NX1", "", "", "e|e,ee,s|es"},
    {"X1N", "", "", "e|e,ee|s|se"},
    {"X1K", "", "s", "e,es|e,ee|s|se"},
    {"XK1", "", "s", "e|e,ee,es|s,se"},
    {"X1K1", "", "s", "e|e,ee,es|s|se"},
    {"X1X", "", "", "e|e,ee,s,es|s|se"},
    {"XX1", "", "", "e|e,ee,s|es,s,se"},
    {"X1X1", "", "", "e|e,ee,s|es,s|se"},
    {"K1N", "s", "", "e|e,ee|se"},
    {"K1K", "s", "s", "e,es|e,ee|se"},
    {"KK1", "s", "s", "e|e,ee,se,es"},
    {"K1K1", "s", "s", "e|e,ee,es|se"},
    {"K1X", "s", "", "e|e,ee,s,es|se"},
    {"KX1", "s", "", "e|e,ee,se,s|es"},
    {"K1X1", "s", "", "e|e,ee,s|se,es"},
    {"I1N", "", "", "e,s|e,ee|se"},
    {"I1K", "", "s", "e,es,s|e,ee|se"},
    {"IK1", "", "s", "e,s|e,ee,se,es"},
    {"I1K1", "", "s", "e,s|e,ee,es|se"},
    {"I1X", "", "", "e,s|e,ee,s,es|se"},
    {"IX1", "", "", "e,s|e,ee,se,s|es"},
    {"I1X1", "", "", "e,s|e,ee,s|se,es"},
};

constexpr const char *kEnumNames[] = {
    "IK", "IN", "IX", "K", "KK", "KN", "KX", "N", "NK", "NN", "NX", "XK", "XN", "XX",
    "NK1", "NX1", "X", "X1K", "XK1", "X1K1", "X1N", "X1X", "XX1", "X1X1", "K1N", "K1K",
    "KK1", "K1K1", "K1X", "KX1", "K1X1", "I1N", "I1K", "IK1", "I1K1", "I1X", "IX1", "I1X1",
    "Npsk0", "Kpsk0", "Xpsk1", "NNpsk0", "NNpsk2", "NKpsk0", "NKpsk2", "NXpsk2", "XNpsk3",
    "XKpsk3", "XXpsk3", "KNpsk0", "KNpsk2", "KKpsk0", "KKpsk2", "KXpsk2", "INpsk1", "INpsk2",
    "IKpsk1", "IKpsk2", "IXpsk2"};
static_assert(sizeof(kEnumNames) / sizeof(kEnumNames[0]) ==
                  (std::size_t)HandshakePattern::IXpsk2 + 1,
              "one name per HandshakePattern");

std::vector<PatternToken> parse_tokens(std::string_view s) {
  std::vector<PatternToken> out;
  std::size_t i = 0;
  while (i < s.size()) {
    std::size_t j = s.find(',', i);
    if (j == std::string_view::npos) j = s.size();
    const std::string_view t = s.substr(i, j - i);
    if (t == "e") out.push_back(PatternToken::E);
    else if (t == "s") out.push_back(PatternToken::S);
    else if (t == "ee") out.push_back(PatternToken::Ee);
    else if (t == "es") out.push_back(PatternToken::Es);
    else if (t == "se") out.push_back(PatternToken::Se);
    else if (t == "ss") out.push_back(PatternToken::Ss);
    else if (t == "psk") out.push_back(PatternToken::Psk);
    else throw std::logic_error("bad pattern token");
    i = j + 1;
  }
  return out;
}
}  // namespace

std::string_view pattern_name(HandshakePattern p) {
  return kEnumNames[(std::size_t)p];
}

namespace detail {
PatternProgram parse_pattern(std::string_view pattern) {
  // base pattern + psk modifiers ("XXpsk0+psk2")
  std::string_view base = pattern;
  std::vector<int> psk_at;
  if (const std::size_t p = pattern.find("psk"); p != std::string_view::npos) {
    base = pattern.substr(0, p);
    std::string_view mods = pattern.substr(p);
    while (!mods.empty()) {
      if (mods.substr(0, 3) != "psk") throw std::logic_error("bad psk modifier");
      std::size_t q = 3;
      int n = 0;
      while (q < mods.size() && mods[q] >= '0' && mods[q] <= '9') n = 10 * n + (mods[q++] - '0');
      if (q == 3) throw std::logic_error("bad psk modifier");
      psk_at.push_back(n);
      mods = mods.substr(q);
      if (!mods.empty()) {
        if (mods[0] != '+') throw std::logic_error("bad psk modifier");
        mods = mods.substr(1);
      }
    }
  }
  const PatternDef *def = nullptr;
  for (const PatternDef &d : kPatterns)
    if (base == d.name) def = &d;
  if (!def) throw std::logic_error("unknown handshake pattern");

  PatternProgram prog;
  prog.pre_i = parse_tokens(def->pre_i);
  prog.pre_r = parse_tokens(def->pre_r);
  for (std::string_view m = def->msgs; !m.empty();) {
    std::size_t j = m.find('|');
    if (j == std::string_view::npos) j = m.size();
    prog.msgs.push_back(parse_tokens(m.substr(0, j)));
    m = j < m.size() ? m.substr(j + 1) : std::string_view();
  }
  for (int n : psk_at) {  // psk0: first token of message 1; pskN: last of message N
    if (n == 0) {
      prog.msgs.front().insert(prog.msgs.front().begin(), PatternToken::Psk);
    } else {
      if ((std::size_t)n > prog.msgs.size()) throw std::logic_error("psk modifier past the last message");
      prog.msgs[n - 1].push_back(PatternToken::Psk);
    }
  }
  prog.npsk = psk_at.size();
  prog.psk_mode = !psk_at.empty();
  prog.one_way = base == "N" || base == "K" || base == "X";
  return prog;
}
}  // namespace detail

}  // namespace noise
