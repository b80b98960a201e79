// transport.cpp -- stream framing and the multi-session batcher over the
// descriptor-batch C ABI (noise_amd/transport.hpp).
#include "noise_amd/transport.hpp"

#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>

#include "noise_gpu.h"

namespace noise::transport {

void append_frame(std::vector<std::uint8_t> &stream, const std::uint8_t *msg, std::size_t len) {
  if (len > kMaxMessage) throw std::length_error("Noise message exceeds 65535 bytes");
  stream.push_back((std::uint8_t)(len >> 8));
  stream.push_back((std::uint8_t)len);
  stream.insert(stream.end(), msg, msg + len);
}

void Deframer::feed(const std::uint8_t *p, std::size_t n) {
  if (pos_ > 0 && pos_ == buf_.size()) {
    buf_.clear();
    pos_ = 0;
  } else if (pos_ > (1u << 20)) {  // compact consumed bytes now and then
    buf_.erase(buf_.begin(), buf_.begin() + (std::ptrdiff_t)pos_);
    pos_ = 0;
  }
  buf_.insert(buf_.end(), p, p + n);
}

bool Deframer::next(std::vector<std::uint8_t> &msg) {
  if (buf_.size() - pos_ < 2) return false;
  const std::size_t len = ((std::size_t)buf_[pos_] << 8) | buf_[pos_ + 1];
  if (buf_.size() - pos_ - 2 < len) return false;
  msg.assign(buf_.begin() + (std::ptrdiff_t)(pos_ + 2), buf_.begin() + (std::ptrdiff_t)(pos_ + 2 + len));
  pos_ += 2 + len;
  return true;
}

std::size_t Batcher::add_session(const CipherState &cs) {
  sessions_.push_back({cs.key_material(), cs.nonce()});
  return sessions_.size() - 1;
}

CipherState Batcher::state(std::size_t s) const {
  const Session &ss = sessions_.at(s);
  CipherState cs;
  cs.initialize_key(ss.k);
  cs.set_nonce(ss.n);
  return cs;
}

void Batcher::submit(std::size_t s, std::vector<std::uint8_t> msg) {
  Session &ss = sessions_.at(s);
  if (ss.n == std::numeric_limits<std::uint64_t>::max() - 1)  // noise.cpp:398-400
    throw std::out_of_range("Nonce limit has been exceeded!");
  if (dir_ == Direction::Encrypt && msg.size() + 16 > kMaxMessage)
    throw std::length_error("Noise message exceeds 65535 bytes");
  if (dir_ == Direction::Decrypt && (msg.size() < 16 || msg.size() > kMaxMessage))
    throw std::invalid_argument("Invalid MAC");  // shorter than a tag
  queue_.push_back({s, ss.n, std::move(msg)});
  ++ss.n;  // decrypt: advances whatever the tag says (noise.cpp:421)
}

std::vector<Batcher::Result> Batcher::flush() {
  std::vector<Result> out;
  if (queue_.empty()) return out;
  const bool dec = dir_ == Direction::Decrypt;
  const std::size_t nrec = queue_.size();
  std::vector<noise_gpu_record> recs(nrec);
  std::uint64_t in_bytes = 0, out_bytes = 0;
  for (std::size_t i = 0; i < nrec; ++i) {  // 16-byte aligned slots: the tile kernels' layout
    const std::uint64_t len = dec ? queue_[i].msg.size() - 16 : queue_[i].msg.size();
    const std::uint64_t in_len = dec ? len + 16 : len, out_len = dec ? len : len + 16;
    recs[i] = noise_gpu_record{in_bytes, out_bytes, queue_[i].nonce, 0, (std::uint32_t)len, 0,
                               (std::uint32_t)queue_[i].session, 0};
    in_bytes += (in_len + 15) / 16 * 16;
    out_bytes += (out_len + 15) / 16 * 16;
  }
  std::vector<std::uint8_t> in(in_bytes ? in_bytes : 1), outb(out_bytes ? out_bytes : 1), st(nrec);
  for (std::size_t i = 0; i < nrec; ++i)
    if (!queue_[i].msg.empty()) std::memcpy(in.data() + recs[i].in_off, queue_[i].msg.data(), queue_[i].msg.size());
  std::vector<std::uint8_t> keys(32 * sessions_.size());
  for (std::size_t s = 0; s < sessions_.size(); ++s) std::memcpy(keys.data() + 32 * s, sessions_[s].k.data(), 32);
  const int rc = dec ? noise_gpu_decrypt_records_host(keys.data(), (std::uint32_t)sessions_.size(), recs.data(),
                                                      nrec, in.data(), in_bytes, outb.data(), out_bytes,
                                                      nullptr, 0, st.data())
                     : noise_gpu_encrypt_records_host(keys.data(), (std::uint32_t)sessions_.size(), recs.data(),
                                                      nrec, in.data(), in_bytes, outb.data(), out_bytes,
                                                      nullptr, 0);
  volatile std::uint8_t *kv = keys.data();
  for (std::size_t i = 0; i < keys.size(); ++i) kv[i] = 0;
  if (rc != NOISE_GPU_OK)
    throw std::runtime_error(std::string("noise-mi355x: ") + noise_gpu_strerror(rc) + ": " +
                             noise_gpu_last_error());
  out.reserve(nrec);
  for (std::size_t i = 0; i < nrec; ++i) {
    Result r{queue_[i].session, queue_[i].nonce, !dec || st[i] == NOISE_GPU_REC_OK, {}};
    const std::size_t olen = dec ? recs[i].len : recs[i].len + 16;
    if (r.ok) r.msg.assign(outb.begin() + (std::ptrdiff_t)recs[i].out_off,
                           outb.begin() + (std::ptrdiff_t)(recs[i].out_off + olen));
    out.push_back(std::move(r));
  }
  queue_.clear();
  return out;
}

}  // namespace noise::transport
