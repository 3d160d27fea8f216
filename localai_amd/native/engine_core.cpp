// Native engine core: paged-KV block manager with a hashed prefix cache, the continuous-batching
// scheduler, and the streaming detokeniser / stop-string matcher.
//
// This is the MI355X-native counterpart of the scheduling half of the reference's C++ backend
// (backend/cpp/llama/grpc-server.cpp: llama_server_context::update_slots :1546-1982, slot
// management :508-557, prompt-prefix reuse common_part :67-74 / :1732-1750, truncation keeping
// n_keep :1694-1720, stop strings + UTF-8 completeness process_token :1010-1123, and the task
// queue in utils.hpp :192-410).  Differences by design:
//   * KV is paged (fixed-size blocks from one global pool sized for 288 GB HBM) instead of a
//     static n_ctx/n_parallel split per slot; prefix reuse is global (hash chain over full
//     blocks) instead of per slot.
//   * Each step packs the device inputs (tokens, positions, slot mapping, block tables, ...)
//     here, so the Python driver only moves ready-made arrays to the GPU.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

#include "text_stream.h"

namespace la {

static inline uint64_t mix64(uint64_t h, uint64_t v) {
  h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 31;
  return h;
}

static uint64_t hash_block(uint64_t parent, const int32_t* toks, int n) {
  uint64_t h = mix64(0xA0761D6478BD642Full, parent);
  for (int i = 0; i < n; ++i) h = mix64(h, (uint64_t)(uint32_t)toks[i]);
  return h;
}

// ------------------------------------------------------------------------------ BlockManager
class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_cache)
      : nb_(num_blocks), bs_(block_size), prefix_(prefix_cache), ref_(num_blocks, 0), hash_(num_blocks, 0),
        hashed_(num_blocks, 0), toks_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("BlockManager: bad sizes");
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }

  int block_size() const { return bs_; }
  int num_blocks() const { return nb_; }
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  int num_cached() const { return (int)map_.size(); }
  int64_t hits() const { return hit_tokens_; }
  int64_t queries() const { return query_tokens_; }

  // Blocks needed to hold n tokens.
  int blocks_for(int n) const { return (n + bs_ - 1) / bs_; }

  // Allocate blocks for a new sequence holding `toks`; returns number of prefix tokens whose KV
  // is already cached (always < toks.size()), or -1 if out of blocks (no side effects).
  int allocate(int64_t sid, const std::vector<int32_t>& toks, int reserve_tokens) {
    if (seqs_.count(sid)) throw std::runtime_error("allocate: sequence exists");
    const int n = (int)toks.size();
    std::vector<int> blocks;
    std::vector<uint64_t> hashes;
    int cached = 0;
    uint64_t h = 0;
    if (prefix_) {
      const int max_full = (n - 1) / bs_;  // never reuse the block holding the last prompt token
      for (int b = 0; b < max_full; ++b) {
        h = hash_block(h, toks.data() + b * bs_, bs_);
        auto it = map_.find(h);
        if (it == map_.end()) break;
        const int blk = it->second;
        if (!std::equal(toks_[blk].begin(), toks_[blk].end(), toks.begin() + b * bs_)) break;
        blocks.push_back(blk);
        hashes.push_back(h);
        cached += bs_;
      }
    }
    const int need = blocks_for(std::max(n, reserve_tokens)) - (int)blocks.size();
    // count availability: cached blocks we are about to reuse may sit in the LRU list
    int reuse_from_lru = 0;
    for (int blk : blocks)
      if (ref_[blk] == 0) ++reuse_from_lru;
    if (need > (int)free_.size() + (int)lru_.size() - reuse_from_lru) return -1;
    for (int blk : blocks) take(blk);
    for (int i = 0; i < need; ++i) blocks.push_back(pop_free());
    Seq s;
    s.blocks = std::move(blocks);
    s.hashes = std::move(hashes);
    s.ntok = cached;
    seqs_.emplace(sid, std::move(s));
    query_tokens_ += n;
    hit_tokens_ += cached;
    return cached;
  }

  // Ensure capacity for `n` total tokens. false if out of blocks.
  bool ensure(int64_t sid, int n) {
    Seq& s = get(sid);
    const int need = blocks_for(n) - (int)s.blocks.size();
    if (need <= 0) return true;
    if (need > num_free()) return false;
    for (int i = 0; i < need; ++i) s.blocks.push_back(pop_free());
    return true;
  }

  int slot(int64_t sid, int pos) {
    Seq& s = get(sid);
    const int b = pos / bs_;
    if (b >= (int)s.blocks.size()) throw std::runtime_error("slot: position beyond allocated blocks");
    return s.blocks[b] * bs_ + (pos % bs_);
  }

  // Mark tokens [0, n) of the sequence as computed; register newly completed full blocks.
  void commit(int64_t sid, const std::vector<int32_t>& toks, int n) {
    Seq& s = get(sid);
    s.ntok = std::max(s.ntok, n);
    if (!prefix_) return;
    const int full = std::min(n, (int)toks.size()) / bs_;
    while ((int)s.hashes.size() < full) {
      const int b = (int)s.hashes.size();
      const uint64_t parent = b ? s.hashes[b - 1] : 0;
      const uint64_t h = hash_block(parent, toks.data() + b * bs_, bs_);
      s.hashes.push_back(h);
      const int blk = s.blocks[b];
      if (!hashed_[blk] && !map_.count(h)) {
        map_[h] = blk;
        hash_[blk] = h;
        hashed_[blk] = 1;
        toks_[blk].assign(toks.begin() + b * bs_, toks.begin() + (b + 1) * bs_);
      }
    }
  }

  void free_seq(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    // release in reverse so the LRU evicts tails before shared prefixes
    for (auto r = it->second.blocks.rbegin(); r != it->second.blocks.rend(); ++r) release(*r);
    seqs_.erase(it);
  }

  std::vector<int> table(int64_t sid) { return get(sid).blocks; }
  bool has(int64_t sid) const { return seqs_.count(sid) > 0; }

  void reset_prefix_cache() {
    for (int blk : lru_) {
      map_.erase(hash_[blk]);
      hashed_[blk] = 0;
      free_.push_back(blk);
    }
    lru_.clear();
    lru_pos_.clear();
  }

 private:
  struct Seq {
    std::vector<int> blocks;
    std::vector<uint64_t> hashes;
    int ntok = 0;
  };
  Seq& get(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence");
    return it->second;
  }
  void take(int blk) {
    if (ref_[blk] == 0) {
      auto it = lru_pos_.find(blk);
      if (it != lru_pos_.end()) {
        lru_.erase(it->second);
        lru_pos_.erase(it);
      }
    }
    ++ref_[blk];
  }
  int pop_free() {
    int blk;
    if (!free_.empty()) {
      blk = free_.back();
      free_.pop_back();
    } else {
      if (lru_.empty()) throw std::runtime_error("out of KV blocks");
      blk = lru_.front();  // evict least recently released cached block
      lru_.pop_front();
      lru_pos_.erase(blk);
      map_.erase(hash_[blk]);
      hashed_[blk] = 0;
    }
    ref_[blk] = 1;
    return blk;
  }
  void release(int blk) {
    if (--ref_[blk] > 0) return;
    if (hashed_[blk]) {
      lru_.push_back(blk);
      lru_pos_[blk] = std::prev(lru_.end());
    } else {
      free_.push_back(blk);
    }
  }

  int nb_, bs_;
  bool prefix_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<uint8_t> hashed_;
  std::vector<std::vector<int32_t>> toks_;
  std::vector<int> free_;
  std::list<int> lru_;
  std::unordered_map<int, std::list<int>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int> map_;
  std::unordered_map<int64_t, Seq> seqs_;
  int64_t hit_tokens_ = 0, query_tokens_ = 0;
};

// ------------------------------------------------------------------------------ Scheduler
struct SeqInfo {
  int64_t id;
  std::vector<int32_t> toks;  // prompt + generated
  int n_prompt = 0;
  int n_computed = 0;  // tokens whose KV is in the cache
  int max_new = 0;
  int n_gen = 0;
  bool running = false;
  int64_t order = 0;
};

class Scheduler {
 public:
  Scheduler(int num_blocks, int block_size, int max_num_seqs, int max_batched_tokens, int max_model_len,
            bool prefix_cache, int decode_bucket_pad)
      : bm_(num_blocks, block_size, prefix_cache), max_seqs_(max_num_seqs), max_tok_(max_batched_tokens),
        max_len_(max_model_len), pad_(decode_bucket_pad) {}

  BlockManager& blocks() { return bm_; }

  void add(int64_t id, std::vector<int32_t> prompt, int max_new) {
    if (prompt.empty()) throw std::invalid_argument("empty prompt");
    if (seqs_.count(id)) throw std::invalid_argument("duplicate sequence id");
    SeqInfo s;
    s.id = id;
    s.n_prompt = (int)prompt.size();
    s.toks = std::move(prompt);
    s.max_new = max_new;
    s.order = counter_++;
    seqs_.emplace(id, std::move(s));
    waiting_.push_back(id);
  }

  // Remove a sequence everywhere (finished, cancelled or failed).
  void finish(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    bm_.free_seq(id);
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    seqs_.erase(it);
  }

  void append(int64_t id, int32_t tok) {
    SeqInfo& s = seqs_.at(id);
    s.toks.push_back(tok);
    s.n_gen++;
  }

  // After a multi-step decode run: `toks` were generated on the device; every one but the last
  // already has its KV written.
  void append_run(int64_t id, const std::vector<int32_t>& toks) {
    SeqInfo& s = seqs_.at(id);
    for (int32_t t : toks) s.toks.push_back(t);
    s.n_gen += (int)toks.size();
    s.n_computed = (int)s.toks.size() - 1;
    bm_.commit(id, s.toks, s.n_computed);
  }

  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  bool has(int64_t id) const { return seqs_.count(id) > 0; }
  int n_gen(int64_t id) const { return seqs_.at(id).n_gen; }
  int n_tokens(int64_t id) const { return (int)seqs_.at(id).toks.size(); }
  std::vector<int32_t> tokens(int64_t id) const { return seqs_.at(id).toks; }

  // lookahead > 1 reserves KV slots for that many decode steps (device-resident multi-step
  // decode: the host comes back only after `lookahead` tokens per sequence).
  // defer_decode: while prompts are waiting or mid-prefill, this step is prefill only (the
  // decode-ready sequences keep their state and reserve nothing) -- the engine asks for it
  // during a request burst, so the burst's prefill chunks run back to back.
  py::dict schedule(int lookahead = 1, bool defer_decode = false) {
    if (lookahead < 1) lookahead = 1;
    if (defer_decode) {
      bool prefill_work = !waiting_.empty() && (int)running_.size() < max_seqs_;
      for (int64_t id : running_) {
        const SeqInfo& s = seqs_.at(id);
        if (!(s.n_computed >= (int)s.toks.size() - 1 && s.n_computed >= s.n_prompt)) prefill_work = true;
      }
      defer_decode = prefill_work;
    }
    std::vector<int64_t> preempted;
    // ---- 1. decode: every running sequence whose prompt is fully computed
    std::vector<int64_t> dec;
    std::vector<int64_t> pre_cont;  // running, still prefilling (chunked)
    // oldest first: when blocks run out, preempt the youngest
    std::sort(running_.begin(), running_.end(),
              [&](int64_t a, int64_t b) { return seqs_.at(a).order < seqs_.at(b).order; });
    for (size_t i = 0; i < running_.size(); ++i) {
      const int64_t id = running_[i];
      SeqInfo& s = seqs_.at(id);
      if (s.n_computed >= (int)s.toks.size() - 1 && s.n_computed >= s.n_prompt) {
        if (defer_decode) continue;
        // needs one new slot for token toks.back() at position toks.size()-1
        while (!bm_.ensure(id, (int)s.toks.size() + lookahead - 1)) {
          // preempt youngest running sequence (recompute later)
          const int64_t victim = running_.back();
          preempt(victim);
          preempted.push_back(victim);
          if (victim == id) break;
        }
        if (!bm_.has(id)) continue;
        dec.push_back(id);
      } else {
        pre_cont.push_back(id);
      }
    }
    // drop preempted from dec / pre_cont
    auto gone = [&](int64_t id) { return !bm_.has(id); };
    dec.erase(std::remove_if(dec.begin(), dec.end(), gone), dec.end());
    pre_cont.erase(std::remove_if(pre_cont.begin(), pre_cont.end(), gone), pre_cont.end());

    // ---- 2. prefill chunks under the token budget
    int budget = max_tok_;
    struct Chunk { int64_t id; int start; int n; };
    std::vector<Chunk> chunks;
    for (int64_t id : pre_cont) {
      if (budget <= 0) break;
      SeqInfo& s = seqs_.at(id);
      const int rem = (int)s.toks.size() - s.n_computed;
      const int n = std::min(rem, budget);
      chunks.push_back({id, s.n_computed, n});
      budget -= n;
    }
    while (!waiting_.empty() && budget > 0 && (int)running_.size() < max_seqs_) {
      const int64_t id = waiting_.front();
      SeqInfo& s = seqs_.at(id);
      const int cached = bm_.allocate(id, s.toks, (int)s.toks.size());
      if (cached < 0) break;  // out of KV blocks: wait for running sequences to finish
      waiting_.pop_front();
      s.n_computed = cached;
      s.running = true;
      running_.push_back(id);
      const int rem = (int)s.toks.size() - cached;
      const int n = std::min(rem, budget);
      chunks.push_back({id, cached, n});
      budget -= n;
    }
    // A deferred (prefill-only) step that found no prefill it can actually run -- the waiting
    // head does not fit the KV pool -- must not come back empty: nothing would decode, so no
    // block would ever be freed and the engine would spin until the prefill-first cap expired.
    // The deferred pass mutated nothing (no decode reservations, no allocation), so plan again
    // with decode.
    if (defer_decode && chunks.empty() && preempted.empty()) return schedule(lookahead, false);

    // ---- 3. pack device inputs
    py::dict out;
    const int bs = bm_.block_size();
    {
      const int np = (int)chunks.size();
      int T = 0, maxb = 1;
      for (auto& c : chunks) {
        T += c.n;
        maxb = std::max(maxb, bm_.blocks_for(c.start + c.n));
      }
      py::array_t<int64_t> ids(np);
      py::array_t<int32_t> tok(T), pos(T), slot(T), cu(np + 1), ctx(np), qlen(np), bt({np, maxb});
      py::array_t<uint8_t> last(np);
      auto* pid = ids.mutable_data();
      auto* pt = tok.mutable_data();
      auto* pp = pos.mutable_data();
      auto* ps = slot.mutable_data();
      auto* pc = cu.mutable_data();
      auto* pctx = ctx.mutable_data();
      auto* pq = qlen.mutable_data();
      auto* pb = bt.mutable_data();
      auto* pl = last.mutable_data();
      int o = 0;
      pc[0] = 0;
      for (int i = 0; i < np; ++i) {
        const Chunk& c = chunks[i];
        SeqInfo& s = seqs_.at(c.id);
        pid[i] = c.id;
        const std::vector<int> tab = bm_.table(c.id);
        for (int j = 0; j < c.n; ++j) {
          const int p = c.start + j;
          pt[o] = s.toks[p];
          pp[o] = p;
          ps[o] = tab[p / bs] * bs + (p % bs);
          ++o;
        }
        pc[i + 1] = o;
        pctx[i] = c.start + c.n;
        pq[i] = c.n;
        pl[i] = (c.start + c.n == (int)s.toks.size()) ? 1 : 0;
        for (int b = 0; b < maxb; ++b) pb[i * maxb + b] = b < (int)tab.size() ? tab[b] : 0;
        s.n_computed = c.start + c.n;
        bm_.commit(c.id, s.toks, s.n_computed);
      }
      out["p_ids"] = ids;
      out["p_tokens"] = tok;
      out["p_pos"] = pos;
      out["p_slots"] = slot;
      out["p_cu"] = cu;
      out["p_ctx"] = ctx;
      out["p_qlen"] = qlen;
      out["p_bt"] = bt;
      out["p_last"] = last;
    }
    {
      const int B = (int)dec.size();
      int Bp = B;
      if (pad_ > 0 && B > 0) Bp = bucket(B);
      int maxb = 1, maxlen = 1;
      for (int64_t id : dec) {
        const int n = (int)seqs_.at(id).toks.size() + lookahead - 1;
        maxb = std::max(maxb, bm_.blocks_for(n));
        maxlen = std::max(maxlen, n);
      }
      py::array_t<int64_t> ids(B);
      py::array_t<int32_t> tok(Bp), pos(Bp), slot(Bp), lens(Bp), bt({Bp, maxb});
      auto* pid = ids.mutable_data();
      auto* pt = tok.mutable_data();
      auto* pp = pos.mutable_data();
      auto* ps = slot.mutable_data();
      auto* pl = lens.mutable_data();
      auto* pb = bt.mutable_data();
      for (int i = 0; i < Bp; ++i) {
        if (i < B) {
          const int64_t id = dec[i];
          SeqInfo& s = seqs_.at(id);
          const int p = (int)s.toks.size() - 1;
          const std::vector<int> tab = bm_.table(id);
          pid[i] = id;
          pt[i] = s.toks[p];
          pp[i] = p;
          ps[i] = tab[p / bs] * bs + (p % bs);
          pl[i] = p + 1;
          for (int b = 0; b < maxb; ++b) pb[i * maxb + b] = b < (int)tab.size() ? tab[b] : 0;
          s.n_computed = p + 1;
          bm_.commit(id, s.toks, s.n_computed);
        } else {  // padding rows: attend to one key of block 0, write no KV
          pt[i] = 0;
          pp[i] = 0;
          ps[i] = -1;
          pl[i] = 1;
          for (int b = 0; b < maxb; ++b) pb[i * maxb + b] = 0;
        }
      }
      out["d_ids"] = ids;
      out["d_tokens"] = tok;
      out["d_pos"] = pos;
      out["d_slots"] = slot;
      out["d_lens"] = lens;
      out["d_bt"] = bt;
      out["d_maxlen"] = maxlen;
    }
    out["preempted"] = preempted;
    return out;
  }

  std::vector<int> buckets() const {
    std::vector<int> v;
    for (int b = 1; b <= max_seqs_; b = next_bucket(b)) v.push_back(b);
    if (v.empty() || v.back() != max_seqs_) v.push_back(max_seqs_);
    return v;
  }

 private:
  static int next_bucket(int b) {
    if (b < 8) return b * 2;
    if (b < 64) return b + 8;
    if (b < 256) return b + 32;
    return b + 64;
  }
  int bucket(int B) const {
    int b = 1;
    while (b < B) b = next_bucket(b);
    return std::min(b, std::max(B, max_seqs_));
  }
  void preempt(int64_t id) {
    SeqInfo& s = seqs_.at(id);
    bm_.free_seq(id);
    s.n_computed = 0;
    s.running = false;
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.push_front(id);
  }

  BlockManager bm_;
  int max_seqs_, max_tok_, max_len_, pad_;
  std::unordered_map<int64_t, SeqInfo> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  int64_t counter_ = 0;
};

// ------------------------------------------------------------------------------ TextStream
// Incremental detokeniser + stop-string matcher (grpc-server.cpp process_token :1010-1123,
// find_partial_stop_string :88-108, UTF-8 completeness :1026-1052).
}  // namespace la

void register_grammar(py::module& m);  // grammar.cpp
void register_http(py::module& m);     // http_server.cpp

PYBIND11_MODULE(_la_core, m) {
  using namespace la;
  register_grammar(m);
  register_http(m);
  m.doc() = "localai_amd native engine core (scheduler, paged KV manager, stop matcher)";
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>())
      .def("allocate", &BlockManager::allocate)
      .def("ensure", &BlockManager::ensure)
      .def("slot", &BlockManager::slot)
      .def("commit", &BlockManager::commit)
      .def("free_seq", &BlockManager::free_seq)
      .def("table", &BlockManager::table)
      .def("has", &BlockManager::has)
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("num_cached", &BlockManager::num_cached)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("hit_tokens", &BlockManager::hits)
      .def_property_readonly("query_tokens", &BlockManager::queries);
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, bool, int>())
      .def("add", &Scheduler::add)
      .def("finish", &Scheduler::finish)
      .def("append", &Scheduler::append)
      .def("schedule", &Scheduler::schedule, py::arg("lookahead") = 1, py::arg("defer_decode") = false)
      .def("append_run", &Scheduler::append_run)
      .def("has", &Scheduler::has)
      .def("n_gen", &Scheduler::n_gen)
      .def("n_tokens", &Scheduler::n_tokens)
      .def("tokens", &Scheduler::tokens)
      .def("buckets", &Scheduler::buckets)
      .def("blocks", &Scheduler::blocks, py::return_value_policy::reference_internal)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running);
  py::class_<Vocab>(m, "Vocab")
      .def(py::init<std::vector<py::bytes>>())
      .def("decode", &Vocab::decode)
      .def("__len__", &Vocab::size);
  py::class_<TextStream>(m, "TextStream")
      .def(py::init<const Vocab*, std::vector<std::string>>(), py::keep_alive<1, 2>())
      .def("push", &TextStream::push)
      .def("push_bytes", &TextStream::push_bytes)
      .def("flush", &TextStream::flush)
      .def("text", &TextStream::text)
      .def_property_readonly("stopped", &TextStream::stopped)
      .def_property_readonly("stop_word", &TextStream::stop_word);
}
