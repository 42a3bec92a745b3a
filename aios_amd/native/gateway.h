// API-gateway core (reference: api-gateway/src/{budget,router}.rs): the monthly
// budget ledger (SQLite, persisted -- the reference kept usage in memory), the response cache
// (sha256(prompt \0 system) keys, TTL, bounded, oldest evicted) and the provider routing policy
// (explicit provider, else claude > openai > qwen3 > local under budget; per-primary fallback
// chains ending at local; JSON mode detection; price table).  The provider HTTP clients stay in
// Python (aiohttp, streaming); every decision and every ledger write is here.
#pragma once
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "json.h"
#include "util.h"

namespace aiosn {

struct GwCompletion {
  std::string text, model_used, provider;
  int64_t tokens_used = 0, latency_ms = 0, input_tokens = 0, output_tokens = 0;
};

class BudgetLedger {
 public:
  BudgetLedger(double claude_budget, double openai_budget, const std::string& db_path = ":memory:");
  // one completion; the 50/50 split of tokens_used when the provider reported no split (the
  // reference's estimate); returns the budget warnings (> 80 % used) it triggers
  std::vector<std::string> record(const std::string& provider, const std::string& model, int64_t tin, int64_t tout,
                                  int64_t tokens_used, double cost_usd, const std::string& agent,
                                  const std::string& task, int64_t now = 0);
  double used(const std::string& provider, int64_t now = 0);  // this billing month
  bool provider_exceeded(const std::string& provider, int64_t now = 0);  // qwen3 / local: never
  bool exceeded(int64_t now = 0);  // both metered providers
  Json status(int64_t now = 0);
  Json usage(const std::string& provider, int days, int64_t now = 0);
  double claude_budget() const { return cb_; }
  double openai_budget() const { return ob_; }
  static int64_t month_start(int64_t unix_seconds);  // UTC

 private:
  void roll(int64_t now);
  double used_locked(const std::string& provider);
  Db db_;
  double cb_, ob_;
  int64_t month_start_ = 0;
  std::mutex mu_;
};

class ResponseCache {
 public:
  explicit ResponseCache(double ttl_s = 3600.0, size_t max_entries = 1000) : ttl_(ttl_s), max_(max_entries) {}
  static std::string key(const std::string& prompt, const std::string& system_prompt);
  std::optional<GwCompletion> get(const std::string& k, double now = 0);
  void put(const std::string& k, const GwCompletion& c, double now = 0);
  size_t size();
  void clear();

 private:
  struct Entry {
    GwCompletion c;
    double at;
    std::list<std::string>::iterator pos;  // insertion order (oldest first)
  };
  double ttl_;
  size_t max_;
  std::unordered_map<std::string, Entry> map_;
  std::list<std::string> order_;
  std::mutex mu_;
};

// routing policy (stateless)
std::string gw_select(const std::string& preferred, const std::map<std::string, bool>& available, BudgetLedger& b,
                      int64_t now = 0);
std::vector<std::string> gw_chain(const std::string& primary, bool allow_fallback);
double gw_cost(const std::string& provider, int64_t tin, int64_t tout);  // USD
bool gw_wants_json(const std::string& prompt, const std::string& system_prompt);

}  // namespace aiosn
