// JSON grammar automaton + vocabulary-trie mask builder -- see grammar.h.
#include "grammar.h"

#include <algorithm>
#include <functional>
#include <map>

namespace aios {

enum JsonMode : uint8_t {
  M_TOP = 0,          // before the top-level value (ws, then '{' or any value)
  M_VALUE,            // expecting a value
  M_OBJ_FIRST,        // after '{': '"' key or '}'
  M_OBJ_KEY,          // after ',' in an object: '"' key
  M_COLON,            // after a key: ':'
  M_ARR_FIRST,        // after '[': value or ']'
  M_AFTER,            // after a value: ',' / closer / (top: done)
  M_STR,              // inside a string
  M_STR_ESC,          // after '\'
  M_STR_U,            // \u + aux hex digits so far
  M_NUM_MINUS,        // '-'
  M_NUM_ZERO,         // leading 0
  M_NUM_INT,          // integer digits
  M_NUM_DOT,          // after '.'
  M_NUM_FRAC,         // fraction digits
  M_NUM_E,            // after e/E
  M_NUM_ESIGN,        // after e+/e-
  M_NUM_EXP,          // exponent digits
  M_LIT,              // inside true/false/null (aux = literal*8 + pos)
  M_DONE,             // complete
};

static const char* kLits[3] = {"true", "false", "null"};

static inline bool is_ws(uint8_t c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; }
static inline bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
static inline bool is_hex(uint8_t c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

static inline bool top_is_obj(const JsonState& s) { return s.depth > 0 && ((s.stack >> (s.depth - 1)) & 1); }

static inline void value_done(JsonState& s) { s.mode = s.depth == 0 ? M_DONE : M_AFTER; }

// start a value with byte c; false if c cannot start a value
static bool start_value(JsonState& s, uint8_t c) {
  switch (c) {
    case '{':
      if (s.depth >= 63) return false;
      s.stack |= (1ULL << s.depth);
      s.depth++;
      s.mode = M_OBJ_FIRST;
      return true;
    case '[':
      if (s.depth >= 63) return false;
      s.stack &= ~(1ULL << s.depth);
      s.depth++;
      s.mode = M_ARR_FIRST;
      return true;
    case '"': s.mode = M_STR; s.in_key = 0; return true;
    case '-': s.mode = M_NUM_MINUS; return true;
    case '0': s.mode = M_NUM_ZERO; return true;
    case 't': s.mode = M_LIT; s.aux = 0 * 8 + 1; return true;
    case 'f': s.mode = M_LIT; s.aux = 1 * 8 + 1; return true;
    case 'n': s.mode = M_LIT; s.aux = 2 * 8 + 1; return true;
    default:
      if (c >= '1' && c <= '9') { s.mode = M_NUM_INT; return true; }
      return false;
  }
}

static bool close_container(JsonState& s, uint8_t c) {
  if (s.depth == 0) return false;
  const bool obj = top_is_obj(s);
  if ((c == '}' && !obj) || (c == ']' && obj)) return false;
  s.depth--;
  s.stack &= ~(1ULL << s.depth);
  value_done(s);
  return true;
}

bool JsonGrammar::step(JsonState& s, uint8_t c, int max_ws) {
  // whitespace between tokens
  auto ws_ok = [&]() {
    if (s.ws >= max_ws) return false;
    s.ws++;
    return true;
  };
  switch (s.mode) {
    case M_TOP:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      return start_value(s, c);
    case M_VALUE:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      return start_value(s, c);
    case M_OBJ_FIRST:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      if (c == '"') { s.mode = M_STR; s.in_key = 1; return true; }
      if (c == '}') return close_container(s, c);
      return false;
    case M_OBJ_KEY:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      if (c == '"') { s.mode = M_STR; s.in_key = 1; return true; }
      return false;
    case M_COLON:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      if (c == ':') { s.mode = M_VALUE; return true; }
      return false;
    case M_ARR_FIRST:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      if (c == ']') return close_container(s, c);
      return start_value(s, c);
    case M_AFTER:
      if (is_ws(c)) return ws_ok();
      s.ws = 0;
      if (c == ',') { s.mode = top_is_obj(s) ? M_OBJ_KEY : M_VALUE; return true; }
      if (c == '}' || c == ']') return close_container(s, c);
      return false;
    case M_STR:
      if (c == '"') {
        if (s.in_key) { s.in_key = 0; s.mode = M_COLON; }
        else value_done(s);
        return true;
      }
      if (c == '\\') { s.mode = M_STR_ESC; return true; }
      return c >= 0x20;  // raw control characters are not allowed in JSON strings
    case M_STR_ESC:
      if (c == 'u') { s.mode = M_STR_U; s.aux = 0; return true; }
      if (c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't') {
        s.mode = M_STR;
        return true;
      }
      return false;
    case M_STR_U:
      if (!is_hex(c)) return false;
      if (++s.aux == 4) { s.mode = M_STR; s.aux = 0; }
      return true;
    case M_NUM_MINUS:
      if (c == '0') { s.mode = M_NUM_ZERO; return true; }
      if (c >= '1' && c <= '9') { s.mode = M_NUM_INT; return true; }
      return false;
    case M_NUM_ZERO:
    case M_NUM_INT:
      if (s.mode == M_NUM_INT && is_digit(c)) return true;
      if (c == '.') { s.mode = M_NUM_DOT; return true; }
      if (c == 'e' || c == 'E') { s.mode = M_NUM_E; return true; }
      value_done(s);
      if (s.mode == M_DONE) return false;  // top-level numbers have no terminator here
      return step(s, c, max_ws);
    case M_NUM_DOT:
      if (is_digit(c)) { s.mode = M_NUM_FRAC; return true; }
      return false;
    case M_NUM_FRAC:
      if (is_digit(c)) return true;
      if (c == 'e' || c == 'E') { s.mode = M_NUM_E; return true; }
      value_done(s);
      if (s.mode == M_DONE) return false;
      return step(s, c, max_ws);
    case M_NUM_E:
      if (c == '+' || c == '-') { s.mode = M_NUM_ESIGN; return true; }
      if (is_digit(c)) { s.mode = M_NUM_EXP; return true; }
      return false;
    case M_NUM_ESIGN:
      if (is_digit(c)) { s.mode = M_NUM_EXP; return true; }
      return false;
    case M_NUM_EXP:
      if (is_digit(c)) return true;
      value_done(s);
      if (s.mode == M_DONE) return false;
      return step(s, c, max_ws);
    case M_LIT: {
      const int li = s.aux >> 3, pos = s.aux & 7;
      const char* lit = kLits[li];
      if ((uint8_t)lit[pos] != c) return false;
      if (lit[pos + 1] == 0) value_done(s);
      else s.aux = (uint8_t)(li * 8 + pos + 1);
      return true;
    }
    case M_DONE:
      return false;
  }
  return false;
}

JsonGrammar::JsonGrammar(const std::vector<std::string>& tokens, int eos_id, int max_ws, bool require_object)
    : tokens_(tokens), eos_(eos_id), max_ws_(max_ws), require_object_(require_object) {
  build_trie();
}

void JsonGrammar::build_trie() {
  // build with maps, then flatten children into edges_ sorted by byte
  struct TmpNode {
    std::map<uint8_t, int> kids;
    std::vector<int> toks;
  };
  std::vector<TmpNode> tmp(1);
  for (int t = 0; t < (int)tokens_.size(); ++t) {
    const std::string& b = tokens_[t];
    if (b.empty()) continue;
    int n = 0;
    for (unsigned char c : b) {
      auto it = tmp[n].kids.find(c);
      if (it == tmp[n].kids.end()) {
        tmp.push_back(TmpNode());
        const int id = (int)tmp.size() - 1;
        tmp[n].kids[c] = id;
        n = id;
      } else {
        n = it->second;
      }
    }
    tmp[n].toks.push_back(t);
  }
  nodes_.resize(tmp.size());
  edges_.clear();
  for (size_t i = 0; i < tmp.size(); ++i) {
    nodes_[i].child_begin = (int)edges_.size();
    nodes_[i].child_count = (int)tmp[i].kids.size();
    for (auto& kv : tmp[i].kids) edges_.push_back({kv.first, kv.second});
    nodes_[i].toks = std::move(tmp[i].toks);
  }
}

JsonState JsonGrammar::initial() const {
  JsonState s;
  s.mode = M_TOP;
  return s;
}

bool JsonGrammar::complete(const JsonState& s) const { return s.mode == M_DONE; }

bool JsonGrammar::accept_bytes(JsonState& s, const std::string& b) const {
  JsonState t = s;
  for (unsigned char c : b) {
    if (require_object_ && t.mode == M_TOP && !is_ws(c) && c != '{') return false;
    if (!step(t, c, max_ws_)) return false;
  }
  s = t;
  return true;
}

bool JsonGrammar::accept_token(JsonState& s, int token) const {
  if (token == eos_) return complete(s);
  if (token < 0 || token >= (int)tokens_.size() || tokens_[token].empty()) return false;
  return accept_bytes(s, tokens_[token]);
}

void JsonGrammar::dfs(int node, JsonState s, std::vector<uint8_t>& out, bool open) const {
  const Node& nd = nodes_[node];
  // open: a token that completes the top-level value is not allowed (min_tokens not reached yet)
  if (!(open && s.mode == M_DONE))
    for (int t : nd.toks) out[t >> 3] |= (uint8_t)(1u << (t & 7));
  for (int e = nd.child_begin; e < nd.child_begin + nd.child_count; ++e) {
    const uint8_t c = edges_[e].first;
    JsonState t = s;
    if (require_object_ && t.mode == M_TOP && !is_ws(c) && c != '{') continue;
    if (!step(t, c, max_ws_)) continue;
    dfs(edges_[e].second, t, out, open);
  }
}

const std::vector<uint8_t>& JsonGrammar::mask(const JsonState& s) {
  auto it = cache_.find(s);
  if (it != cache_.end()) return it->second;
  if (cache_.size() > 8192) cache_.clear();
  std::vector<uint8_t> m((tokens_.size() + 7) / 8, 0);
  if (complete(s)) {
    if (eos_ >= 0 && eos_ < (int)tokens_.size()) m[eos_ >> 3] |= (uint8_t)(1u << (eos_ & 7));
  } else {
    dfs(0, s, m);
  }
  return cache_.emplace(s, std::move(m)).first->second;
}

const std::vector<uint8_t>& JsonGrammar::mask_open(const JsonState& s) {
  if (complete(s)) return mask(s);
  auto it = cache_open_.find(s);
  if (it != cache_open_.end()) return it->second;
  if (cache_open_.size() > 8192) cache_open_.clear();
  std::vector<uint8_t> m((tokens_.size() + 7) / 8, 0);
  dfs(0, s, m, true);
  bool any = false;
  for (uint8_t b : m) any |= b != 0;
  if (!any) return mask(s);  // only closing tokens are left: the value may complete
  return cache_open_.emplace(s, std::move(m)).first->second;
}

}  // namespace aios
