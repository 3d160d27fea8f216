// Detokenising text stream with stop-string hold-back and UTF-8 completeness (shared by the
// engine core and the native HTTP token sinks).
#pragma once
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace la {

class Vocab {
 public:
  explicit Vocab(std::vector<py::bytes> pieces) {
    pieces_.reserve(pieces.size());
    for (auto& p : pieces) pieces_.push_back(std::string(p));
  }
  const std::string& piece(int32_t t) const {
    static const std::string empty;
    if (t < 0 || t >= (int32_t)pieces_.size()) return empty;
    return pieces_[t];
  }
  size_t size() const { return pieces_.size(); }
  py::bytes decode(const std::vector<int32_t>& toks) const {
    std::string s;
    for (int32_t t : toks) s += piece(t);
    return py::bytes(s);
  }

 private:
  std::vector<std::string> pieces_;
};

static int utf8_incomplete_tail(const std::string& s) {
  // number of trailing bytes that form an incomplete UTF-8 sequence
  const int n = (int)s.size();
  for (int i = 1; i <= std::min(4, n); ++i) {
    const unsigned char c = (unsigned char)s[n - i];
    if ((c & 0xC0) == 0x80) continue;  // continuation byte
    int need = 0;
    if ((c & 0xE0) == 0xC0) need = 2;
    else if ((c & 0xF0) == 0xE0) need = 3;
    else if ((c & 0xF8) == 0xF0) need = 4;
    else return 0;  // ASCII or invalid lead: complete
    return (i < need) ? i : 0;
  }
  return 0;
}

class TextStream {
 public:
  TextStream(const Vocab* vocab, std::vector<std::string> stops) : v_(vocab), stops_(std::move(stops)) {
    for (auto& s : stops_) maxstop_ = std::max(maxstop_, s.size());
  }
  // Feed one token; returns (bytes safe to emit now, stop hit)
  py::tuple push(int32_t tok) {
    auto r = push_raw(tok);
    return py::make_tuple(py::bytes(r.first), r.second);
  }
  py::tuple push_bytes(const std::string& b) {
    buf_ += b;
    auto r = drain();
    return py::make_tuple(py::bytes(r.first), r.second);
  }
  std::pair<std::string, bool> push_raw(int32_t tok) {
    buf_ += v_->piece(tok);
    return drain();
  }
  std::string flush_raw() {
    std::string out = buf_;
    buf_.clear();
    all_ += out;
    return out;
  }
  // flush everything held back (end of generation)
  py::bytes flush() {
    std::string out = buf_;
    buf_.clear();
    all_ += out;
    return py::bytes(out);
  }
  py::bytes text() const { return py::bytes(all_); }
  bool stopped() const { return stopped_; }
  std::string stop_word() const { return stop_word_; }

 private:
  std::pair<std::string, bool> drain() {
    if (stopped_) return {std::string(), true};
    // full stop-string match anywhere in the pending buffer
    size_t best = std::string::npos;
    for (auto& s : stops_) {
      if (s.empty()) continue;
      const size_t p = buf_.find(s);
      if (p != std::string::npos && p < best) {
        best = p;
        stop_word_ = s;
      }
    }
    if (best != std::string::npos) {
      std::string out = buf_.substr(0, best);
      all_ += out;
      buf_.clear();
      stopped_ = true;
      return {out, true};
    }
    // hold back the longest suffix that is a proper prefix of some stop string
    size_t hold = 0;
    for (auto& s : stops_) {
      const size_t m = std::min(s.size() - 1, buf_.size());
      for (size_t l = m; l > hold; --l) {
        if (buf_.compare(buf_.size() - l, l, s, 0, l) == 0) {
          hold = l;
          break;
        }
      }
    }
    const std::string head = buf_.substr(0, buf_.size() - hold);
    const int inc = utf8_incomplete_tail(head);
    const size_t emit = head.size() - inc;
    std::string out = buf_.substr(0, emit);
    buf_.erase(0, emit);
    all_ += out;
    return {out, false};
  }

  const Vocab* v_;
  std::vector<std::string> stops_;
  size_t maxstop_ = 0;
  std::string buf_, all_, stop_word_;
  bool stopped_ = false;
};

}  // namespace la
