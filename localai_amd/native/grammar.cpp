// GBNF grammar-constrained decoding (the reference uses llama.cpp's llama-grammar.cpp through
// grpc-server.cpp; grammars come from pkg/functions/grammars and the `grammar` request field).
//
// Grammar  : GBNF text -> flat rule tables (literals, char classes, rule refs; `*`, `+`, `?` and
//            `{m,n}` are rewritten into helper rules).
// State    : a set of pushdown stacks (pointers into the rule tables) plus a pending partial
//            UTF-8 code point.  accept(token) feeds the token's code points through the stacks.
// filter() : decides a batch of candidate tokens at once without mutating the state; the engine
//            asks it only for the device sampler's top candidates (the device produces logits and
//            the top-N, the host PDA keeps the first accepted ones), falling back to a whole-
//            vocabulary scan over a byte trie when none of them is accepted.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace lagr {

enum ET : uint8_t { END = 0, ALT, RULE_REF, CHAR, CHAR_NOT, CHAR_RNG_UPPER, CHAR_ALT, CHAR_ANY };
struct El {
  ET type;
  uint32_t value;
};
using Rule = std::vector<El>;

static inline bool is_end(const El* e) { return e->type == END || e->type == ALT; }

// ------------------------------------------------------------------------------------ parser
class Parser {
 public:
  std::vector<Rule> rules;
  std::map<std::string, uint32_t> ids;

  explicit Parser(const std::string& src) : s_(src) {}

  void parse() {
    size_t p = skip(0, true);
    while (p < s_.size()) p = parse_rule(p);
    for (size_t i = 0; i < rules.size(); ++i) {
      if (rules[i].empty()) {
        std::string name = "?";
        for (auto& kv : ids)
          if (kv.second == i) name = kv.first;
        throw std::invalid_argument("grammar: undefined rule '" + name + "'");
      }
      for (auto& e : rules[i])
        if (e.type == RULE_REF && (e.value >= rules.size() || rules[e.value].empty()))
          throw std::invalid_argument("grammar: reference to an undefined rule");
    }
  }

  uint32_t sym(const std::string& name) {
    auto it = ids.find(name);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)ids.size();
    ids[name] = id;
    return id;
  }

 private:
  const std::string& s_;
  int gen_ = 0;

  [[noreturn]] void fail(size_t p, const char* what) {
    throw std::invalid_argument(std::string("grammar parse error: ") + what + " at offset " + std::to_string(p));
  }
  static bool is_word(char c) { return isalnum((unsigned char)c) || c == '-' || c == '_'; }

  size_t skip(size_t p, bool newline_ok) {
    while (p < s_.size()) {
      const char c = s_[p];
      if (c == ' ' || c == '\t') {
        ++p;
      } else if (c == '#') {
        while (p < s_.size() && s_[p] != '\n' && s_[p] != '\r') ++p;
      } else if (newline_ok && (c == '\n' || c == '\r')) {
        ++p;
      } else {
        break;
      }
    }
    return p;
  }

  size_t parse_name(size_t p, std::string& out) {
    const size_t b = p;
    while (p < s_.size() && is_word(s_[p])) ++p;
    if (p == b) fail(p, "expected a name");
    out = s_.substr(b, p - b);
    return p;
  }

  uint32_t decode_utf8(size_t& p) {
    const unsigned char c = (unsigned char)s_[p];
    int n = 1;
    uint32_t v = c;
    if (c >= 0xF0) { n = 4; v = c & 0x07; }
    else if (c >= 0xE0) { n = 3; v = c & 0x0F; }
    else if (c >= 0xC0) { n = 2; v = c & 0x1F; }
    ++p;
    for (int i = 1; i < n && p < s_.size(); ++i, ++p) v = (v << 6) | ((unsigned char)s_[p] & 0x3F);
    return v;
  }

  uint32_t parse_hex(size_t& p, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i, ++p) {
      if (p >= s_.size()) fail(p, "truncated escape");
      const char c = s_[p];
      int d;
      if (c >= '0' && c <= '9') d = c - '0';
      else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
      else fail(p, "bad hex escape");
      v = v * 16 + (uint32_t)d;
    }
    return v;
  }

  uint32_t parse_char(size_t& p) {
    if (p >= s_.size()) fail(p, "unexpected end");
    if (s_[p] == '\\') {
      ++p;
      if (p >= s_.size()) fail(p, "unexpected end of escape");
      const char c = s_[p++];
      switch (c) {
        case 'x': return parse_hex(p, 2);
        case 'u': return parse_hex(p, 4);
        case 'U': return parse_hex(p, 8);
        case 't': return '\t';
        case 'r': return '\r';
        case 'n': return '\n';
        case '\\': case '"': case '[': case ']': case '-': case '^': return (uint32_t)c;
        default: fail(p, "unknown escape");
      }
    }
    return decode_utf8(p);
  }

  size_t parse_rule(size_t p) {
    std::string name;
    p = parse_name(p, name);
    p = skip(p, false);
    if (s_.compare(p, 3, "::=") != 0) fail(p, "expected ::=");
    p = skip(p + 3, true);
    const uint32_t id = sym(name);
    Rule r;
    p = parse_alternates(p, name, r, false);
    if (rules.size() <= id) rules.resize(id + 1);
    rules[id] = std::move(r);
    if (p < s_.size() && s_[p] == '\r') ++p;
    if (p < s_.size() && s_[p] == '\n') ++p;
    return skip(p, true);
  }

  size_t parse_alternates(size_t p, const std::string& name, Rule& out, bool nested) {
    p = parse_sequence(p, name, out, nested);
    while (p < s_.size() && s_[p] == '|') {
      out.push_back({ALT, 0});
      p = parse_sequence(skip(p + 1, true), name, out, nested);
    }
    out.push_back({END, 0});
    return p;
  }

  uint32_t new_rule(const std::string& base, Rule&& r) {
    const uint32_t id = sym(base + "_" + std::to_string(gen_++));
    if (rules.size() <= id) rules.resize(id + 1);
    rules[id] = std::move(r);
    return id;
  }

  size_t parse_sequence(size_t p, const std::string& name, Rule& out, bool nested) {
    size_t last_start = out.size();
    while (p < s_.size()) {
      const char c = s_[p];
      if (c == '"') {
        ++p;
        last_start = out.size();
        while (p < s_.size() && s_[p] != '"') out.push_back({CHAR, parse_char(p)});
        if (p >= s_.size()) fail(p, "unterminated literal");
        p = skip(p + 1, nested);
      } else if (c == '[') {
        ++p;
        ET start = CHAR;
        if (p < s_.size() && s_[p] == '^') {
          start = CHAR_NOT;
          ++p;
        }
        last_start = out.size();
        while (p < s_.size() && s_[p] != ']') {
          const uint32_t ch = parse_char(p);
          out.push_back({out.size() > last_start ? CHAR_ALT : start, ch});
          if (p + 1 < s_.size() && s_[p] == '-' && s_[p + 1] != ']') {
            ++p;
            out.push_back({CHAR_RNG_UPPER, parse_char(p)});
          }
        }
        if (p >= s_.size()) fail(p, "unterminated char class");
        if (out.size() == last_start) out.push_back({start, 0});  // "[]" / "[^]" edge
        p = skip(p + 1, nested);
      } else if (is_word(c)) {
        std::string ref;
        p = parse_name(p, ref);
        last_start = out.size();
        out.push_back({RULE_REF, sym(ref)});
        p = skip(p, nested);
      } else if (c == '(') {
        Rule sub;
        p = parse_alternates(skip(p + 1, true), name, sub, true);
        if (p >= s_.size() || s_[p] != ')') fail(p, "expected )");
        last_start = out.size();
        out.push_back({RULE_REF, new_rule(name, std::move(sub))});
        p = skip(p + 1, nested);
      } else if (c == '.') {
        last_start = out.size();
        out.push_back({CHAR_ANY, 0});
        p = skip(p + 1, nested);
      } else if (c == '*' || c == '+' || c == '?' || c == '{') {
        if (last_start == out.size()) fail(p, "repetition without a preceding item");
        int mn = 0, mx = -1;
        if (c == '*') { mn = 0; mx = -1; ++p; }
        else if (c == '+') { mn = 1; mx = -1; ++p; }
        else if (c == '?') { mn = 0; mx = 1; ++p; }
        else {
          ++p;
          size_t b = p;
          while (p < s_.size() && isdigit((unsigned char)s_[p])) ++p;
          if (p == b) fail(p, "expected a number in {m,n}");
          mn = std::stoi(s_.substr(b, p - b));
          if (p < s_.size() && s_[p] == ',') {
            ++p;
            b = p;
            while (p < s_.size() && isdigit((unsigned char)s_[p])) ++p;
            mx = (p == b) ? -1 : std::stoi(s_.substr(b, p - b));
          } else {
            mx = mn;
          }
          if (p >= s_.size() || s_[p] != '}') fail(p, "expected }");
          ++p;
        }
        Rule item(out.begin() + (long)last_start, out.end());
        out.resize(last_start);
        repeat(name, item, mn, mx, out);
        p = skip(p, nested);
      } else {
        break;
      }
    }
    return p;
  }

  // out += item{mn} then (mx - mn) optional copies (or a star rule when mx == -1)
  void repeat(const std::string& name, const Rule& item, int mn, int mx, Rule& out) {
    for (int i = 0; i < mn; ++i) out.insert(out.end(), item.begin(), item.end());
    if (mx == -1) {
      // R ::= item R | eps
      const uint32_t id = sym(name + "_" + std::to_string(gen_++));
      if (rules.size() <= id) rules.resize(id + 1);
      Rule r(item);
      r.push_back({RULE_REF, id});
      r.push_back({ALT, 0});
      r.push_back({END, 0});
      rules[id] = std::move(r);
      out.push_back({RULE_REF, id});
      return;
    }
    // nested optionals: R_k ::= item R_{k-1} | eps  (built innermost first)
    uint32_t inner = UINT32_MAX;
    for (int k = 0; k < mx - mn; ++k) {
      Rule r(item);
      if (inner != UINT32_MAX) r.push_back({RULE_REF, inner});
      r.push_back({ALT, 0});
      r.push_back({END, 0});
      inner = new_rule(name, std::move(r));
    }
    if (inner != UINT32_MAX) out.push_back({RULE_REF, inner});
  }
};

class Grammar {
 public:
  Grammar(const std::string& text, const std::string& root) {
    Parser ps(text);
    ps.parse();
    auto it = ps.ids.find(root);
    if (it == ps.ids.end()) throw std::invalid_argument("grammar: no '" + root + "' rule");
    rules = std::move(ps.rules);
    root_id = it->second;
    n_named = 0;
    for (auto& kv : ps.ids) names[kv.second] = kv.first;
  }
  std::vector<Rule> rules;
  uint32_t root_id;
  int n_named;
  std::unordered_map<uint32_t, std::string> names;
  size_t num_rules() const { return rules.size(); }
};

using Stack = std::vector<const El*>;

static void advance_stack(const std::vector<Rule>& rules, const Stack& st, std::vector<Stack>& out, int depth = 0) {
  if (depth > 2048) throw std::runtime_error("grammar: left recursion or nesting too deep");
  if (st.empty()) {
    if (std::find(out.begin(), out.end(), st) == out.end()) out.push_back(st);
    return;
  }
  const El* pos = st.back();
  if (pos->type == RULE_REF) {
    const El* sub = rules[pos->value].data();
    for (;;) {
      Stack ns(st.begin(), st.end() - 1);
      if (!is_end(pos + 1)) ns.push_back(pos + 1);
      if (!is_end(sub)) ns.push_back(sub);
      advance_stack(rules, ns, out, depth + 1);
      while (!is_end(sub)) ++sub;
      if (sub->type == ALT) ++sub;
      else break;
    }
    return;
  }
  if (std::find(out.begin(), out.end(), st) == out.end()) out.push_back(st);
}

// does the char element group at pos accept code point c?  -> element after the group
static bool match_char(const El* pos, uint32_t c, const El** after) {
  if (pos->type == CHAR_ANY) {
    *after = pos + 1;
    return true;
  }
  const bool positive = pos->type == CHAR;
  bool found = false;
  do {
    if (pos[1].type == CHAR_RNG_UPPER) {
      found = found || (pos->value <= c && c <= pos[1].value);
      pos += 2;
    } else {
      found = found || pos->value == c;
      pos += 1;
    }
  } while (pos->type == CHAR_ALT);
  *after = pos;
  return found == positive;
}

static void accept_char(const std::vector<Rule>& rules, const std::vector<Stack>& in, uint32_t c,
                        std::vector<Stack>& out) {
  out.clear();
  for (const Stack& st : in) {
    if (st.empty()) continue;
    const El* after;
    if (!match_char(st.back(), c, &after)) continue;
    Stack ns(st.begin(), st.end() - 1);
    if (!is_end(after)) ns.push_back(after);
    advance_stack(rules, ns, out);
  }
}

// UTF-8 decoder that carries a partial code point across tokens
struct Utf8 {
  uint32_t value = 0;
  int remain = 0;
  uint32_t min = 0;  // smallest code point the sequence may encode (rejects overlong forms)
};

static bool feed_bytes(const std::vector<Rule>& rules, std::vector<Stack>& stacks, Utf8& u, const std::string& b,
                       std::vector<Stack>& tmp) {
  for (unsigned char c : b) {
    if (u.remain > 0) {
      if ((c & 0xC0) != 0x80) return false;
      u.value = (u.value << 6) | (c & 0x3F);
      if (--u.remain > 0) continue;
      if (u.value < u.min || u.value > 0x10FFFF || (u.value >= 0xD800 && u.value <= 0xDFFF)) return false;
    } else if (c < 0x80) {
      u.value = c;
    } else if (c >= 0xC2 && c <= 0xDF) {
      u.value = c & 0x1F; u.remain = 1; u.min = 0x80; continue;
    } else if ((c & 0xF0) == 0xE0) {
      u.value = c & 0x0F; u.remain = 2; u.min = 0x800; continue;
    } else if (c >= 0xF0 && c <= 0xF4) {
      u.value = c & 0x07; u.remain = 3; u.min = 0x10000; continue;
    } else {
      return false;  // stray continuation byte, overlong lead (C0/C1) or > U+10FFFF
    }
    accept_char(rules, stacks, u.value, tmp);
    stacks.swap(tmp);
    if (stacks.empty()) return false;
  }
  return true;
}

// can some completion of a partial code point (value v, n bytes missing) be accepted by any stack?
static bool partial_ok(const std::vector<Stack>& stacks, const Utf8& u) {
  if (u.remain == 0) return !stacks.empty();
  const uint32_t low = std::max(u.value << (6 * u.remain), u.min);
  const uint32_t high = (u.value << (6 * u.remain)) | ((1u << (6 * u.remain)) - 1);
  if (low > high) return false;
  for (const Stack& st : stacks) {
    if (st.empty()) continue;
    const El* pos = st.back();
    if (pos->type == CHAR_ANY) return true;
    const bool positive = pos->type == CHAR;
    bool overlap = false, covered = false;
    do {
      uint32_t a = pos->value, b = pos->value;
      if (pos[1].type == CHAR_RNG_UPPER) {
        b = pos[1].value;
        pos += 2;
      } else {
        pos += 1;
      }
      if (a <= high && low <= b) overlap = true;
      if (a <= low && high <= b) covered = true;
    } while (pos->type == CHAR_ALT);
    if (positive ? overlap : !covered) return true;
  }
  return false;
}

// Byte trie over the vocabulary's token pieces: node 0 is the root; `toks` are the tokens whose
// piece ends at the node.  The whole-vocabulary mask walks it depth-first, feeding one byte per
// edge, so a prefix the grammar rejects prunes every token below it at once.
struct TrieNode {
  std::vector<std::pair<uint8_t, int>> kids;
  std::vector<int32_t> toks;
};

class GrammarVocab {
 public:
  explicit GrammarVocab(std::vector<py::bytes> pieces, std::vector<int32_t> eog) : eog_(eog.begin(), eog.end()) {
    pieces_.reserve(pieces.size());
    for (auto& p : pieces) pieces_.push_back(std::string(p));
    trie_.emplace_back();
    for (size_t t = 0; t < pieces_.size(); ++t) {
      const std::string& b = pieces_[t];
      if (b.empty() || is_eog((int)t)) continue;
      int node = 0;
      for (unsigned char c : b) {
        int next = -1;
        for (auto& kv : trie_[node].kids)
          if (kv.first == c) { next = kv.second; break; }
        if (next < 0) {
          next = (int)trie_.size();
          trie_[node].kids.emplace_back(c, next);
          trie_.emplace_back();
        }
        node = next;
      }
      trie_[node].toks.push_back((int32_t)t);
    }
  }
  const std::vector<TrieNode>& trie() const { return trie_; }
  const std::vector<int32_t>& eog_list() const { return eog_; }
  const std::string& piece(int t) const {
    static const std::string empty;
    return (t >= 0 && t < (int)pieces_.size()) ? pieces_[t] : empty;
  }
  bool is_eog(int t) const { return std::find(eog_.begin(), eog_.end(), t) != eog_.end(); }
  size_t size() const { return pieces_.size(); }

 private:
  std::vector<std::string> pieces_;
  std::vector<int32_t> eog_;
  std::vector<TrieNode> trie_;
};

class GrammarState {
 public:
  GrammarState(std::shared_ptr<Grammar> g, std::shared_ptr<GrammarVocab> v) : g_(std::move(g)), v_(std::move(v)) {
    const Rule& root = g_->rules[g_->root_id];
    const El* alt = root.data();
    for (;;) {
      Stack st;
      if (!is_end(alt)) st.push_back(alt);
      advance_stack(g_->rules, st, stacks_);
      while (!is_end(alt)) ++alt;
      if (alt->type == ALT) ++alt;
      else break;
    }
  }

  bool can_end() const {
    if (u_.remain) return false;
    for (auto& s : stacks_)
      if (s.empty()) return true;
    return false;
  }

  bool check_piece(const std::string& b) const {
    if (b.empty()) return false;
    std::vector<Stack> st = stacks_, tmp;
    Utf8 u = u_;
    return feed_bytes(g_->rules, st, u, b, tmp) && partial_ok(st, u);
  }

  bool check(int tok) const {
    if (v_->is_eog(tok)) return can_end();
    return check_piece(v_->piece(tok));
  }

  // accepted flags for a batch of candidate tokens (state unchanged)
  py::array_t<uint8_t> filter(py::array_t<int32_t, py::array::c_style | py::array::forcecast> cand) const {
    const auto n = cand.size();
    py::array_t<uint8_t> out(n);
    auto* o = out.mutable_data();
    const int32_t* c = cand.data();
    py::gil_scoped_release rel;
    for (py::ssize_t i = 0; i < n; ++i) o[i] = check(c[i]) ? 1 : 0;
    return out;
  }

  // whole-vocabulary mask: depth-first over the byte trie (same decisions as check() per token)
  py::array_t<uint8_t> mask() const {
    const size_t V = v_->size();
    py::array_t<uint8_t> out(V);
    auto* o = out.mutable_data();
    py::gil_scoped_release rel;
    std::fill(o, o + V, 0);
    const bool end_ok = can_end();
    for (int32_t t : v_->eog_list())
      if (t >= 0 && (size_t)t < V) o[t] = end_ok ? 1 : 0;
    trie_walk(0, stacks_, u_, o);
    return out;
  }

  // reference implementation: one check() per token (tests compare the two)
  py::array_t<uint8_t> mask_linear() const {
    const size_t V = v_->size();
    py::array_t<uint8_t> out(V);
    auto* o = out.mutable_data();
    py::gil_scoped_release rel;
    for (size_t t = 0; t < V; ++t) o[t] = check((int)t) ? 1 : 0;
    return out;
  }

  // whole-vocabulary mask with a bound on the trie edges fed: None when the walk would exceed
  // `budget` (a permissive state, e.g. inside a JSON string, where most of the vocabulary is
  // allowed and the full walk costs tens of ms); restrictive states finish far below it
  py::object mask_limited(long budget) const {
    const size_t V = v_->size();
    py::array_t<uint8_t> out(V);
    auto* o = out.mutable_data();
    bool ok;
    {
      py::gil_scoped_release rel;
      std::fill(o, o + V, 0);
      const bool end_ok = can_end();
      for (int32_t t : v_->eog_list())
        if (t >= 0 && (size_t)t < V) o[t] = end_ok ? 1 : 0;
      long left = budget;
      ok = trie_walk(0, stacks_, u_, o, &left);
    }
    if (!ok) return py::none();
    return std::move(out);
  }

  // identity of the parse state for mask caching: FNV-1a over the sorted per-stack hashes (stack
  // order depends on history, the set does not) and the partial UTF-8 code point
  uint64_t key() const { return key_of(stacks_, u_, done_); }

  // the key of the state after each candidate token (0: the token is rejected, or ends the
  // grammar), without changing this state -- one level of the parse-state transition graph
  py::array_t<uint64_t> next_keys(py::array_t<int32_t, py::array::c_style | py::array::forcecast> cand) const {
    const auto n = cand.size();
    py::array_t<uint64_t> out(n);
    auto* o = out.mutable_data();
    const int32_t* c = cand.data();
    py::gil_scoped_release rel;
    std::vector<Stack> st, tmp;
    for (py::ssize_t i = 0; i < n; ++i) {
      o[i] = 0;
      if (v_->is_eog(c[i])) continue;
      const std::string& b = v_->piece(c[i]);
      if (b.empty()) continue;
      st = stacks_;
      Utf8 u = u_;
      if (!feed_bytes(g_->rules, st, u, b, tmp)) continue;
      o[i] = key_of(st, u, false);
      if (o[i] == 0) o[i] = 1;
    }
    return out;
  }

  static uint64_t key_of(const std::vector<Stack>& stacks, const Utf8& u, bool done) {
    std::vector<uint64_t> hs;
    hs.reserve(stacks.size());
    for (const Stack& st : stacks) {
      uint64_t h = 1469598103934665603ull;
      for (const El* e : st) {
        h ^= (uint64_t)(uintptr_t)e;
        h *= 1099511628211ull;
      }
      h ^= st.size();
      h *= 1099511628211ull;
      hs.push_back(h);
    }
    std::sort(hs.begin(), hs.end());
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](uint64_t x) {
      for (int i = 0; i < 8; ++i) {
        h ^= (x >> (8 * i)) & 0xFF;
        h *= 1099511628211ull;
      }
    };
    for (uint64_t x : hs) mix(x);
    // the decoder keeps the last code point in `value` after it completes: only a pending
    // partial code point is part of the state
    mix(u.remain ? u.value : 0);
    mix(u.remain ? (((uint64_t)u.remain << 32) | u.min) : 0);
    mix(done ? 1 : 0);
    return h;
  }

  bool trie_walk(int node, const std::vector<Stack>& stacks, const Utf8& u, uint8_t* o, long* left = nullptr) const {
    const auto& trie = v_->trie();
    std::vector<Stack> st, tmp;
    for (const auto& kv : trie[node].kids) {
      if (left && --*left < 0) return false;
      st = stacks;
      Utf8 uu = u;
      const std::string one(1, (char)kv.first);
      if (!feed_bytes(g_->rules, st, uu, one, tmp)) continue;  // rejected prefix: prune the subtree
      const TrieNode& child = trie[kv.second];
      if (!child.toks.empty() && partial_ok(st, uu))
        for (int32_t t : child.toks) o[t] = 1;
      if (!child.kids.empty() && !trie_walk(kv.second, st, uu, o, left)) return false;
    }
    return true;
  }

  bool accept(int tok) {
    if (v_->is_eog(tok)) {
      if (!can_end()) return false;
      done_ = true;
      return true;
    }
    const std::string& b = v_->piece(tok);
    if (b.empty()) return false;
    std::vector<Stack> st = stacks_, tmp;
    Utf8 u = u_;
    if (!feed_bytes(g_->rules, st, u, b, tmp)) return false;
    stacks_.swap(st);
    u_ = u;
    return true;
  }

  bool accept_bytes(const std::string& b) {
    std::vector<Stack> st = stacks_, tmp;
    Utf8 u = u_;
    if (!feed_bytes(g_->rules, st, u, b, tmp)) return false;
    stacks_.swap(st);
    u_ = u;
    return true;
  }

  size_t num_stacks() const { return stacks_.size(); }
  bool done() const { return done_; }

 private:
  std::shared_ptr<Grammar> g_;
  std::shared_ptr<GrammarVocab> v_;
  std::vector<Stack> stacks_;
  Utf8 u_;
  bool done_ = false;
};

}  // namespace lagr

void register_grammar(py::module& m) {
  using namespace lagr;
  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "Grammar")
      .def(py::init<const std::string&, const std::string&>(), py::arg("text"), py::arg("root") = "root")
      .def_property_readonly("num_rules", &Grammar::num_rules);
  py::class_<GrammarVocab, std::shared_ptr<GrammarVocab>>(m, "GrammarVocab")
      .def(py::init<std::vector<py::bytes>, std::vector<int32_t>>())
      .def("__len__", &GrammarVocab::size);
  py::class_<GrammarState>(m, "GrammarState")
      .def(py::init<std::shared_ptr<Grammar>, std::shared_ptr<GrammarVocab>>())
      .def("check", &GrammarState::check)
      .def("check_bytes", &GrammarState::check_piece)
      .def("filter", &GrammarState::filter)
      .def("mask", &GrammarState::mask)
      .def("mask_linear", &GrammarState::mask_linear)
      .def("mask_limited", &GrammarState::mask_limited, py::arg("budget"))
      .def("key", &GrammarState::key)
      .def("next_keys", &GrammarState::next_keys)
      .def("clone", [](const GrammarState& s) { return GrammarState(s); })
      .def("accept", &GrammarState::accept)
      .def("accept_bytes", &GrammarState::accept_bytes)
      .def("can_end", &GrammarState::can_end)
      .def_property_readonly("num_stacks", &GrammarState::num_stacks)
      .def_property_readonly("done", &GrammarState::done);
}
