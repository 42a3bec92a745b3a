// API-gateway core: budget ledger, response cache, routing policy (see gateway.h).
// Reference behaviour: api-gateway/src/budget.rs (monthly $100 Claude / $50 OpenAI, 80 % warning,
// monthly reset), router.rs:34-248 (cache TTL 3600 s, 1000 entries, oldest evicted; claude >
// openai > qwen3 > local; fallback chains), openai.rs:137 (JSON mode trigger).
#include "gateway.h"

#include <algorithm>
#include <chrono>
#include <ctime>

namespace aiosn {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}
int64_t or_now(int64_t t) { return t > 0 ? t : now_unix(); }
}  // namespace

// ------------------------------------------------------------------------------------ ledger
int64_t BudgetLedger::month_start(int64_t t) {
  const time_t tt = (time_t)t;
  struct tm tm;
  gmtime_r(&tt, &tm);
  tm.tm_mday = 1;
  tm.tm_hour = tm.tm_min = tm.tm_sec = 0;
  return (int64_t)timegm(&tm);
}

BudgetLedger::BudgetLedger(double claude_budget, double openai_budget, const std::string& db_path)
    : db_(db_path), cb_(claude_budget), ob_(openai_budget) {
  db_.exec(
      "CREATE TABLE IF NOT EXISTS usage (provider TEXT, model TEXT, input_tokens INTEGER, output_tokens INTEGER,"
      " cost_usd REAL, timestamp INTEGER, requesting_agent TEXT, task_id TEXT)");
  db_.exec("CREATE INDEX IF NOT EXISTS usage_pt ON usage(provider, timestamp)");
  month_start_ = month_start(now_unix());
}

// the billing month of `now` (the counters restart on the 1st, UTC; records are kept)
void BudgetLedger::roll(int64_t now) { month_start_ = month_start(now); }

double BudgetLedger::used_locked(const std::string& provider) {
  std::lock_guard<std::recursive_mutex> g(db_.mutex());
  Stmt s(db_, "SELECT COALESCE(SUM(cost_usd), 0) FROM usage WHERE provider = ? AND timestamp >= ?");
  s.bind(1, provider).bind(2, month_start_);
  return s.step() ? s.col_double(0) : 0.0;
}

std::vector<std::string> BudgetLedger::record(const std::string& provider, const std::string& model, int64_t tin,
                                              int64_t tout, int64_t tokens_used, double cost_usd,
                                              const std::string& agent, const std::string& task, int64_t now) {
  now = or_now(now);
  if (tin == 0 && tout == 0 && tokens_used) {
    tin = tokens_used / 2;
    tout = tokens_used - tokens_used / 2;
  }
  std::lock_guard<std::mutex> g(mu_);
  roll(now);
  {
    std::lock_guard<std::recursive_mutex> dg(db_.mutex());
    Stmt s(db_, "INSERT INTO usage VALUES (?,?,?,?,?,?,?,?)");
    s.bind(1, provider).bind(2, model).bind(3, tin).bind(4, tout).bind(5, cost_usd).bind(6, now).bind(7, agent).bind(8,
                                                                                                                 task);
    s.exec();
  }
  std::vector<std::string> warn;
  const std::pair<const char*, double> metered[] = {{"claude", cb_}, {"openai", ob_}};
  for (auto& m : metered) {
    const double u = used_locked(m.first);
    if (m.second > 0 && u > 0.8 * m.second) {
      char buf[160];
      snprintf(buf, sizeof buf, "%s budget warning: $%.2f / $%.2f (%d%%)", m.first, u, m.second,
               (int)(100.0 * u / m.second));
      warn.emplace_back(buf);
    }
  }
  return warn;
}

double BudgetLedger::used(const std::string& provider, int64_t now) {
  std::lock_guard<std::mutex> g(mu_);
  roll(or_now(now));
  return used_locked(provider);
}

bool BudgetLedger::provider_exceeded(const std::string& provider, int64_t now) {
  if (provider != "claude" && provider != "openai") return false;  // qwen3 / local are not metered
  const double u = used(provider, now);
  return u >= (provider == "claude" ? cb_ : ob_);
}

bool BudgetLedger::exceeded(int64_t now) { return provider_exceeded("claude", now) && provider_exceeded("openai", now); }

Json BudgetLedger::status(int64_t now) {
  now = or_now(now);
  const double cu = used("claude", now), ou = used("openai", now);
  const time_t tt = (time_t)now;
  struct tm tm;
  gmtime_r(&tt, &tm);
  const int day = tm.tm_mday;
  Json j = Json::object();
  j.set("claude_monthly_budget_usd", cb_);
  j.set("claude_used_usd", cu);
  j.set("openai_monthly_budget_usd", ob_);
  j.set("openai_used_usd", ou);
  j.set("days_remaining", (int64_t)std::max(0, 30 - day));
  j.set("daily_rate_usd", (cu + ou) / std::max(day, 1));
  j.set("budget_exceeded", cu >= cb_ && ou >= ob_);
  return j;
}

Json BudgetLedger::usage(const std::string& provider, int days, int64_t now) {
  now = or_now(now);
  const int64_t cutoff = days > 0 ? now - (int64_t)days * 86400 : 0;
  std::string q =
      "SELECT provider, model, input_tokens, output_tokens, cost_usd, timestamp, requesting_agent, task_id FROM usage "
      "WHERE timestamp >= ?";
  if (!provider.empty()) q += " AND provider = ?";
  q += " ORDER BY timestamp, rowid";
  Json recs = Json::array();
  double total = 0;
  int64_t toks = 0, n = 0;
  {
    std::lock_guard<std::recursive_mutex> g(db_.mutex());
    Stmt s(db_, q);
    s.bind(1, cutoff);
    if (!provider.empty()) s.bind(2, provider);
    while (s.step()) {
      Json r = Json::object();
      r.set("provider", s.col_text(0));
      r.set("model", s.col_text(1));
      r.set("input_tokens", s.col_int(2));
      r.set("output_tokens", s.col_int(3));
      r.set("cost_usd", s.col_double(4));
      r.set("timestamp", s.col_int(5));
      r.set("requesting_agent", s.col_text(6));
      r.set("task_id", s.col_text(7));
      total += s.col_double(4);
      toks += s.col_int(2) + s.col_int(3);
      ++n;
      recs.push(r);
    }
  }
  Json j = Json::object();
  j.set("records", recs);
  j.set("total_cost_usd", total);
  j.set("total_requests", n);
  j.set("total_tokens", toks);
  return j;
}

// ------------------------------------------------------------------------------------ cache
std::string ResponseCache::key(const std::string& prompt, const std::string& system_prompt) {
  std::string m;
  m.reserve(prompt.size() + system_prompt.size() + 1);
  m += prompt;
  m.push_back('\0');
  m += system_prompt;
  return sha256_hex(m);
}

std::optional<GwCompletion> ResponseCache::get(const std::string& k, double now) {
  if (now <= 0) now = now_s();
  std::lock_guard<std::mutex> g(mu_);
  auto it = map_.find(k);
  if (it == map_.end()) return std::nullopt;
  if (now - it->second.at >= ttl_) {  // expired
    order_.erase(it->second.pos);
    map_.erase(it);
    return std::nullopt;
  }
  return it->second.c;
}

void ResponseCache::put(const std::string& k, const GwCompletion& c, double now) {
  if (now <= 0) now = now_s();
  std::lock_guard<std::mutex> g(mu_);
  auto it = map_.find(k);
  if (it != map_.end()) {  // refresh: moves to the newest end
    order_.erase(it->second.pos);
    map_.erase(it);
  } else if (max_ > 0 && map_.size() >= max_) {  // full: evict the oldest insertion
    map_.erase(order_.front());
    order_.pop_front();
  }
  order_.push_back(k);
  map_.emplace(k, Entry{c, now, std::prev(order_.end())});
}

size_t ResponseCache::size() {
  std::lock_guard<std::mutex> g(mu_);
  return map_.size();
}

void ResponseCache::clear() {
  std::lock_guard<std::mutex> g(mu_);
  map_.clear();
  order_.clear();
}

// ------------------------------------------------------------------------------------ routing
std::string gw_select(const std::string& preferred, const std::map<std::string, bool>& available, BudgetLedger& b,
                      int64_t now) {
  if (!preferred.empty()) return preferred;
  for (const char* p : {"claude", "openai", "qwen3"}) {
    auto it = available.find(p);
    if (it != available.end() && it->second && !b.provider_exceeded(p, now)) return p;
  }
  return "local";
}

std::vector<std::string> gw_chain(const std::string& primary, bool allow_fallback) {
  std::vector<std::string> c{primary};
  if (!allow_fallback) return c;
  static const std::map<std::string, std::vector<std::string>> fb = {
      {"claude", {"openai", "qwen3", "local"}},
      {"openai", {"claude", "qwen3", "local"}},
      {"qwen3", {"claude", "openai", "local"}},
      {"local", {"qwen3", "claude", "openai"}},
  };
  auto it = fb.find(primary);
  if (it == fb.end()) c.push_back("local");
  else c.insert(c.end(), it->second.begin(), it->second.end());
  return c;
}

double gw_cost(const std::string& provider, int64_t tin, int64_t tout) {
  double pin = 0, pout = 0;  // USD per 1M tokens
  if (provider == "claude") { pin = 3.0; pout = 15.0; }
  else if (provider == "openai") { pin = 2.5; pout = 10.0; }
  return (double)tin * pin / 1e6 + (double)tout * pout / 1e6;
}

bool gw_wants_json(const std::string& prompt, const std::string& system_prompt) {
  return contains(prompt, "valid JSON") || contains(prompt, "JSON object") ||
         contains(system_prompt, "respond with ONLY valid JSON");
}

}  // namespace aiosn
