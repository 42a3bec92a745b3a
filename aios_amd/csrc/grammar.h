// JSON-mode constrained decoding.
//
// The reference always asks llama-server for `response_format: {"type":"json_object"}`
// (`runtime/src/inference.rs:119-121`), i.e. grammar-constrained generation of one JSON object.
// Here: a byte-level JSON pushdown recogniser whose whole state is a 16-byte POD (container
// stack as a 64-bit bitmask), a trie over the vocabulary's byte strings, and a DFS that carries
// the POD state down the trie to produce the allowed-token bitmask for the current state (pruned
// at the first rejected byte), memoised per state.  The mask is applied on device by the sampler
// kernel (aios::SampleArgs::mask).
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace aios {

struct JsonState {
  uint64_t stack = 0;   // bit i: container at depth i is an object (1) or array (0)
  uint8_t depth = 0;
  uint8_t mode = 0;     // see JsonMode
  uint8_t aux = 0;      // literal index / unicode digit count
  uint8_t ws = 0;       // consecutive whitespace (capped)
  uint8_t in_key = 0;   // current string is an object key
  uint8_t pad[3] = {0, 0, 0};
  bool operator==(const JsonState& o) const {
    return stack == o.stack && depth == o.depth && mode == o.mode && aux == o.aux && ws == o.ws && in_key == o.in_key;
  }
};

struct JsonStateHash {
  size_t operator()(const JsonState& s) const {
    uint64_t h = s.stack * 0x9E3779B97F4A7C15ULL;
    h ^= ((uint64_t)s.depth << 40) ^ ((uint64_t)s.mode << 32) ^ ((uint64_t)s.aux << 24) ^ ((uint64_t)s.ws << 16) ^
         ((uint64_t)s.in_key << 8);
    return (size_t)(h ^ (h >> 29));
  }
};

class JsonGrammar {
 public:
  // tokens: byte string of every vocabulary entry (empty for control tokens)
  JsonGrammar(const std::vector<std::string>& tokens, int eos_id, int max_ws = 20, bool require_object = true);

  JsonState initial() const;
  static bool step(JsonState& s, uint8_t c, int max_ws);  // false = byte rejected
  bool accept_token(JsonState& s, int token) const;       // applies the token (no-op + false on reject)
  bool accept_bytes(JsonState& s, const std::string& b) const;
  bool complete(const JsonState& s) const;                // a full top-level value has been produced
  // allowed-token bitmask (ceil(V/8) bytes, bit i of byte t/8 set = token t allowed)
  const std::vector<uint8_t>& mask(const JsonState& s);
  // the same without the tokens that complete the top-level value (falls back to mask() when
  // nothing else is allowed): a request's min_tokens keeps the object open until it is reached
  const std::vector<uint8_t>& mask_open(const JsonState& s);
  int vocab_size() const { return (int)tokens_.size(); }
  size_t cache_size() const { return cache_.size(); }

 private:
  struct Node {
    int child_begin = 0;  // index into edges_
    int child_count = 0;
    std::vector<int> toks;
  };
  void build_trie();
  void dfs(int node, JsonState s, std::vector<uint8_t>& out, bool open = false) const;

  std::vector<std::string> tokens_;
  int eos_;
  int max_ws_;
  bool require_object_;
  std::vector<Node> nodes_;
  std::vector<std::pair<uint8_t, int>> edges_;  // (byte, child node)
  std::unordered_map<JsonState, std::vector<uint8_t>, JsonStateHash> cache_;
  std::unordered_map<JsonState, std::vector<uint8_t>, JsonStateHash> cache_open_;
};

}  // namespace aios
