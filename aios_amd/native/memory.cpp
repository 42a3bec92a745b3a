#include "memory.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <queue>
#include <set>
#include <unordered_map>

namespace aiosn {

// ------------------------------------------------------------------------------ embedding
std::vector<float> hashed_embedding(const std::string& text, int dim) {
  // bag of words (alnum runs, > 2 chars, lowercased); two buckets per word: h % dim (+count) and
  // (h >> 16) % dim (+0.5 count), h = fold(h*31 + byte); L2-normalised   (longterm.rs:14-50)
  std::vector<float> v((size_t)dim, 0.f);
  std::unordered_map<std::string, int> counts;
  std::string w;
  auto flush = [&]() {
    if (w.size() > 2) counts[w]++;
    w.clear();
  };
  for (unsigned char c : text) {
    if (std::isalnum(c) || c >= 0x80) w += (char)std::tolower(c);
    else flush();
  }
  flush();
  if (counts.empty()) return v;
  for (auto& kv : counts) {
    uint64_t h = 0;
    for (unsigned char b : kv.first) h = h * 31 + b;
    v[h % (uint64_t)dim] += (float)kv.second;
    v[(h >> 16) % (uint64_t)dim] += 0.5f * (float)kv.second;
  }
  double n = 0;
  for (float x : v) n += (double)x * x;
  n = std::sqrt(n);
  if (n > 0)
    for (auto& x : v) x = (float)(x / n);
  return v;
}

double cosine(const std::vector<float>& a, const std::vector<float>& b) {
  if (a.size() != b.size() || a.empty()) return 0;
  double d = 0, na = 0, nb = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    d += (double)a[i] * b[i];
    na += (double)a[i] * a[i];
    nb += (double)b[i] * b[i];
  }
  return (na > 0 && nb > 0) ? d / std::sqrt(na * nb) : 0;
}

double keyword_relevance(const std::vector<std::string>& kws, const std::string& text) {
  if (kws.empty()) return 0.5;
  const std::string t = lower(text);
  int m = 0;
  for (auto& k : kws)
    if (t.find(lower(k)) != std::string::npos) ++m;
  return (double)m / (double)kws.size();
}

int estimate_tokens(const std::string& s) { return (int)((s.size() + 3) / 4); }

// ---- collection scans: the query side is prepared once, every row is scored without allocating, and only
// the top-n rows are materialised as records (a scan used to build a record for every row, then sort them all)
namespace {
struct Scorer {
  std::vector<std::string> kws;  // lower-cased once
  std::vector<float> qe;
  explicit Scorer(const std::string& query) : qe(hashed_embedding(query)) {
    for (auto& k : split_ws(query)) kws.push_back(lower(k));
  }
  // 0.4 * keyword overlap + 0.6 * cosine(query, stored embedding blob)   (longterm.rs:186)
  double operator()(const std::string& text, const std::string& emb) const {
    double kw = 0.5;
    if (!kws.empty()) {
      const std::string t = lower(text);
      int m = 0;
      for (auto& k : kws)
        if (t.find(k) != std::string::npos) ++m;
      kw = (double)m / (double)kws.size();
    }
    double cos = 0;
    const size_t n = emb.size() / 4;
    if (n == qe.size() && n) {
      double d = 0, na = 0, nb = 0;
      for (size_t i = 0; i < n; ++i) {
        float b;
        std::memcpy(&b, emb.data() + 4 * i, 4);
        d += (double)qe[i] * b;
        na += (double)qe[i] * qe[i];
        nb += (double)b * b;
      }
      cos = (na > 0 && nb > 0) ? d / std::sqrt(na * nb) : 0;
    }
    return 0.4 * kw + 0.6 * cos;
  }
};

// the n best (relevance desc, scan order on ties -- what a stable sort of every row gave)
class TopN {
 public:
  explicit TopN(int n) : n_((size_t)std::max(n, 0)) {}
  bool wants(double r) const { return n_ && (heap_.size() < n_ || r > heap_.top().r); }
  void push(double r, Json rec) {
    heap_.push({r, seq_++, std::move(rec)});
    if (heap_.size() > n_) heap_.pop();
  }
  void skip() { ++seq_; }
  Json take() {
    std::vector<Hit> v;
    while (!heap_.empty()) {
      v.push_back(std::move(const_cast<Hit&>(heap_.top())));
      heap_.pop();
    }
    Json out = Json::array();
    for (auto it = v.rbegin(); it != v.rend(); ++it) out.push(std::move(it->rec));
    return out;
  }

 private:
  struct Hit {
    double r;
    size_t seq;
    Json rec;
  };
  struct Worse {  // heap top = the current worst kept hit
    bool operator()(const Hit& a, const Hit& b) const { return a.r != b.r ? a.r > b.r : a.seq < b.seq; }
  };
  size_t n_, seq_ = 0;
  std::priority_queue<Hit, std::vector<Hit>, Worse> heap_;
};
}  // namespace

static std::string emb_blob(const std::vector<float>& v) { return std::string((const char*)v.data(), v.size() * 4); }
static std::vector<float> blob_emb(const std::string& b) {
  std::vector<float> v(b.size() / 4);
  if (!v.empty()) std::memcpy(v.data(), b.data(), v.size() * 4);
  return v;
}
// proto3 defaults ("" / 0) mean "unset": fill ids and timestamps
static std::string id_of(const Json& j) {
  const std::string id = j.get_str("id");
  return id.empty() ? uuid4() : id;
}
static int64_t ts_of(const Json& j, const char* k) {
  const int64_t t = j.get_int(k);
  return t ? t : now_unix();
}
static std::string bytes_of(const Json& j, const char* k) {
  const Json& v = j[k];
  return v.is_str() ? v.as_str() : (v.is_null() ? "" : v.dump());
}

// ------------------------------------------------------------------------------ operational
void OperationalMemory::push_event(Json ev) {
  if (ev.get_str("id").empty()) ev.set("id", uuid4());
  if (ev.get_int("timestamp") == 0) ev.set("timestamp", now_unix());
  std::lock_guard<std::mutex> g(mu_);
  events_.push_back(std::move(ev));
  while (events_.size() > cap_) events_.pop_front();
}
Json OperationalMemory::recent(int count, const std::string& category, const std::string& source) const {
  std::lock_guard<std::mutex> g(mu_);
  Json out = Json::array();
  if (count <= 0) count = 10;
  for (auto it = events_.rbegin(); it != events_.rend() && (int)out.size() < count; ++it) {
    if (!category.empty() && it->get_str("category") != category) continue;
    if (!source.empty() && it->get_str("source") != source) continue;
    out.push(*it);
  }
  return out;
}
void OperationalMemory::update_metric(const std::string& key, double value, int64_t ts) {
  std::lock_guard<std::mutex> g(mu_);
  metrics_[key] = {value, ts ? ts : now_unix()};
}
bool OperationalMemory::metric(const std::string& key, double& value, int64_t& ts) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = metrics_.find(key);
  if (it == metrics_.end()) return false;
  value = it->second.first;
  ts = it->second.second;
  return true;
}
Json OperationalMemory::snapshot() const {
  // metric keys of operational.rs:63-82
  std::lock_guard<std::mutex> g(mu_);
  auto m = [&](const char* k) {
    auto it = metrics_.find(k);
    return it == metrics_.end() ? 0.0 : it->second.first;
  };
  Json models = Json::array();
  for (auto& kv : metrics_)
    if (starts_with(kv.first, "model.loaded.") && kv.second.first > 0) models.push(kv.first.substr(13));
  return Json::object({{"cpu_percent", m("cpu.usage")},
                       {"memory_used_mb", m("memory.used_mb")},
                       {"memory_total_mb", m("memory.total_mb")},
                       {"disk_used_gb", m("disk.used_gb")},
                       {"disk_total_gb", m("disk.total_gb")},
                       {"gpu_utilization", m("gpu.utilization")},
                       {"active_tasks", (int64_t)m("tasks.active")},
                       {"active_agents", (int64_t)m("agents.active")},
                       {"loaded_models", models}});
}
size_t OperationalMemory::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return events_.size();
}

// ------------------------------------------------------------------------------ store
MemoryStore::MemoryStore(const std::string& wdb, const std::string& ldb, const std::string& kdb)
    : work_(wdb), lt_(ldb), kn_(kdb) {
  work_.exec(
      "CREATE TABLE IF NOT EXISTS goals (id TEXT PRIMARY KEY, description TEXT, status TEXT, priority INTEGER,"
      " created_at INTEGER, completed_at INTEGER, result TEXT, metadata_json TEXT);"
      "CREATE TABLE IF NOT EXISTS tasks (id TEXT PRIMARY KEY, goal_id TEXT, description TEXT, agent TEXT, status TEXT,"
      " input_json TEXT, output_json TEXT, started_at INTEGER, completed_at INTEGER, duration_ms INTEGER, error TEXT);"
      "CREATE INDEX IF NOT EXISTS idx_tasks_goal ON tasks(goal_id);"
      "CREATE TABLE IF NOT EXISTS tool_calls (id TEXT PRIMARY KEY, task_id TEXT, tool_name TEXT, agent TEXT,"
      " input_json TEXT, output_json TEXT, success INTEGER, duration_ms INTEGER, reason TEXT, timestamp INTEGER);"
      "CREATE INDEX IF NOT EXISTS idx_calls_task ON tool_calls(task_id);"
      "CREATE TABLE IF NOT EXISTS decisions (id TEXT PRIMARY KEY, context TEXT, options_json TEXT, chosen TEXT,"
      " reasoning TEXT, intelligence_level TEXT, model_used TEXT, outcome TEXT, timestamp INTEGER);"
      "CREATE TABLE IF NOT EXISTS patterns (id TEXT PRIMARY KEY, trigger TEXT, action TEXT, success_rate REAL,"
      " uses INTEGER, last_used INTEGER, created_from TEXT);"
      "CREATE TABLE IF NOT EXISTS agent_states (agent_name TEXT PRIMARY KEY, state_json TEXT, updated_at INTEGER);");
  lt_.exec(
      "CREATE TABLE IF NOT EXISTS procedures (id TEXT PRIMARY KEY, name TEXT, description TEXT, steps_json TEXT,"
      " success_count INTEGER, fail_count INTEGER, avg_duration_ms INTEGER, tags TEXT, created_at INTEGER,"
      " last_used INTEGER, embedding BLOB);"
      "CREATE TABLE IF NOT EXISTS incidents (id TEXT PRIMARY KEY, description TEXT, symptoms_json TEXT, root_cause TEXT,"
      " resolution TEXT, resolved_by TEXT, prevention TEXT, timestamp INTEGER, embedding BLOB);"
      "CREATE TABLE IF NOT EXISTS config_changes (id TEXT PRIMARY KEY, file_path TEXT, content TEXT, changed_by TEXT,"
      " reason TEXT, timestamp INTEGER);");
  kn_.exec(
      "CREATE TABLE IF NOT EXISTS knowledge (id TEXT PRIMARY KEY, title TEXT, content TEXT, source TEXT, tags TEXT,"
      " created_at INTEGER, embedding BLOB);");
}

// ---- working
void MemoryStore::store_goal(const Json& g) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO goals VALUES (?1,?2,?3,?4,?5,?6,?7,?8)");
  s.bind(1, id_of(g)).bind(2, g.get_str("description")).bind(3, g.get_str("status", "pending"));
  s.bind(4, g.get_int("priority", 5)).bind(5, ts_of(g, "created_at")).bind(6, g.get_int("completed_at"));
  s.bind(7, g.get_str("result")).bind(8, bytes_of(g, "metadata_json")).exec();
}
void MemoryStore::update_goal(const std::string& id, const std::string& status, const std::string& result) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  const bool done = status == "completed" || status == "failed" || status == "cancelled";
  Stmt s(work_, "UPDATE goals SET status = ?2, result = CASE WHEN ?3 = '' THEN result ELSE ?3 END,"
                " completed_at = CASE WHEN ?4 > 0 THEN ?4 ELSE completed_at END WHERE id = ?1");
  s.bind(1, id).bind(2, status).bind(3, result).bind(4, done ? now_unix() : (int64_t)0).exec();
}
static Json goal_row(Stmt& s) {
  return Json::object({{"id", s.col_text(0)}, {"description", s.col_text(1)}, {"status", s.col_text(2)},
                       {"priority", s.col_int(3)}, {"created_at", s.col_int(4)}, {"completed_at", s.col_int(5)},
                       {"result", s.col_text(6)}, {"metadata_json", s.col_text(7)}});
}
Json MemoryStore::active_goals() {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "SELECT * FROM goals WHERE status IN ('pending','in_progress','active','awaiting_input')"
                " ORDER BY priority ASC, created_at DESC");
  Json out = Json::array();
  while (s.step()) out.push(goal_row(s));
  return out;
}
void MemoryStore::store_task(const Json& t) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO tasks VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9,?10,?11)");
  s.bind(1, id_of(t)).bind(2, t.get_str("goal_id")).bind(3, t.get_str("description"));
  s.bind(4, t.get_str("agent")).bind(5, t.get_str("status", "pending")).bind(6, bytes_of(t, "input_json"));
  s.bind(7, bytes_of(t, "output_json")).bind(8, t.get_int("started_at")).bind(9, t.get_int("completed_at"));
  s.bind(10, t.get_int("duration_ms")).bind(11, t.get_str("error")).exec();
}
Json MemoryStore::tasks_for_goal(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "SELECT * FROM tasks WHERE goal_id = ?1 ORDER BY started_at ASC");
  s.bind(1, goal_id);
  Json out = Json::array();
  while (s.step())
    out.push(Json::object({{"id", s.col_text(0)}, {"goal_id", s.col_text(1)}, {"description", s.col_text(2)},
                           {"agent", s.col_text(3)}, {"status", s.col_text(4)}, {"input_json", s.col_text(5)},
                           {"output_json", s.col_text(6)}, {"started_at", s.col_int(7)}, {"completed_at", s.col_int(8)},
                           {"duration_ms", s.col_int(9)}, {"error", s.col_text(10)}}));
  return out;
}
void MemoryStore::store_tool_call(const Json& c) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO tool_calls VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9,?10)");
  s.bind(1, id_of(c)).bind(2, c.get_str("task_id")).bind(3, c.get_str("tool_name"));
  s.bind(4, c.get_str("agent")).bind(5, bytes_of(c, "input_json")).bind(6, bytes_of(c, "output_json"));
  s.bind(7, (int64_t)c.get_bool("success")).bind(8, c.get_int("duration_ms")).bind(9, c.get_str("reason"));
  s.bind(10, ts_of(c, "timestamp")).exec();
}
void MemoryStore::store_decision(const Json& d) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO decisions VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9)");
  s.bind(1, id_of(d)).bind(2, d.get_str("context")).bind(3, bytes_of(d, "options_json"));
  s.bind(4, d.get_str("chosen")).bind(5, d.get_str("reasoning")).bind(6, d.get_str("intelligence_level"));
  s.bind(7, d.get_str("model_used")).bind(8, d.get_str("outcome")).bind(9, ts_of(d, "timestamp")).exec();
}
void MemoryStore::store_pattern(const Json& p) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO patterns VALUES (?1,?2,?3,?4,?5,?6,?7)");
  s.bind(1, id_of(p)).bind(2, p.get_str("trigger")).bind(3, p.get_str("action"));
  s.bind(4, p.get_num("success_rate", 1.0)).bind(5, p.get_int("uses")).bind(6, ts_of(p, "last_used"));
  s.bind(7, p.get_str("created_from")).exec();
}
Json MemoryStore::find_pattern(const std::string& trigger, double min_success) {
  // LIKE %trigger%, best success rate then most uses (working.rs:306-340)
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "SELECT id, trigger, action, success_rate, uses, last_used, created_from FROM patterns"
                " WHERE (trigger LIKE ?1 OR ?2 LIKE '%' || trigger || '%') AND success_rate >= ?3"
                " ORDER BY success_rate DESC, uses DESC LIMIT 1");
  s.bind(1, "%" + trigger + "%").bind(2, trigger).bind(3, min_success);
  if (!s.step()) return Json::object();
  return Json::object({{"id", s.col_text(0)}, {"trigger", s.col_text(1)}, {"action", s.col_text(2)},
                       {"success_rate", s.col_double(3)}, {"uses", s.col_int(4)}, {"last_used", s.col_int(5)},
                       {"created_from", s.col_text(6)}});
}
void MemoryStore::update_pattern_stats(const std::string& id, bool success) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "UPDATE patterns SET success_rate = (success_rate * uses + ?2) / (uses + 1), uses = uses + 1,"
                " last_used = ?3 WHERE id = ?1");
  s.bind(1, id).bind(2, success ? 1.0 : 0.0).bind(3, now_unix()).exec();
}
void MemoryStore::store_agent_state(const std::string& agent, const std::string& state_json) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "INSERT OR REPLACE INTO agent_states VALUES (?1,?2,?3)");
  s.bind(1, agent).bind(2, state_json).bind(3, now_unix()).exec();
}
Json MemoryStore::agent_state(const std::string& agent) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "SELECT agent_name, state_json, updated_at FROM agent_states WHERE agent_name = ?1");
  s.bind(1, agent);
  if (!s.step()) return Json::object({{"agent_name", agent}, {"state_json", ""}, {"updated_at", 0}});
  return Json::object({{"agent_name", s.col_text(0)}, {"state_json", s.col_text(1)}, {"updated_at", s.col_int(2)}});
}
Json MemoryStore::tool_sequence_for_goal(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt s(work_, "SELECT c.tool_name, c.success FROM tool_calls c JOIN tasks t ON c.task_id = t.id"
                " WHERE t.goal_id = ?1 ORDER BY c.timestamp ASC");
  s.bind(1, goal_id);
  Json out = Json::array();
  while (s.step()) out.push(Json::object({{"tool", s.col_text(0)}, {"success", s.col_int(1) != 0}}));
  return out;
}
Json MemoryStore::learn_pattern_from_goal(const std::string& goal_id) {
  // working.rs:377-426: a completed goal's successful tool sequence becomes a reusable pattern
  std::lock_guard<std::recursive_mutex> l(work_.mutex());
  Stmt g(work_, "SELECT description, status FROM goals WHERE id = ?1");
  g.bind(1, goal_id);
  if (!g.step()) return Json::object();
  const std::string desc = g.col_text(0), status = g.col_text(1);
  if (status != "completed") return Json::object();
  Json seq = tool_sequence_for_goal(goal_id);
  Json tools = Json::array();
  for (auto& c : seq.as_arr())
    if (c.get_bool("success")) tools.push(c.get_str("tool"));
  if (!tools.size()) return Json::object();
  // trigger: the goal's leading keywords
  auto words = split_ws(lower(desc));
  std::string trig;
  for (size_t i = 0; i < words.size() && i < 6; ++i) trig += (trig.empty() ? "" : " ") + words[i];
  Json p = Json::object({{"id", uuid4()}, {"trigger", trig}, {"action", tools.dump()}, {"success_rate", 1.0},
                         {"uses", 1}, {"last_used", now_unix()}, {"created_from", goal_id}});
  store_pattern(p);
  return p;
}

// ---- long-term
void MemoryStore::store_procedure(const Json& p) {
  std::lock_guard<std::recursive_mutex> l(lt_.mutex());
  std::string tags;
  for (auto& t : p["tags"].as_arr()) tags += (tags.empty() ? "" : ",") + t.as_str();
  const auto emb = hashed_embedding(p.get_str("name") + " " + p.get_str("description") + " " + tags);
  Stmt s(lt_, "INSERT OR REPLACE INTO procedures VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9,?10,?11)");
  s.bind(1, id_of(p)).bind(2, p.get_str("name")).bind(3, p.get_str("description"));
  s.bind(4, bytes_of(p, "steps_json")).bind(5, p.get_int("success_count")).bind(6, p.get_int("fail_count"));
  s.bind(7, p.get_int("avg_duration_ms")).bind(8, tags).bind(9, ts_of(p, "created_at"));
  s.bind(10, ts_of(p, "last_used"));
  const std::string b = emb_blob(emb);
  s.bind_blob(11, b.data(), b.size()).exec();
}
void MemoryStore::store_incident(const Json& i) {
  std::lock_guard<std::recursive_mutex> l(lt_.mutex());
  const auto emb = hashed_embedding(i.get_str("description") + " " + i.get_str("root_cause") + " " + i.get_str("resolution"));
  Stmt s(lt_, "INSERT OR REPLACE INTO incidents VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9)");
  s.bind(1, id_of(i)).bind(2, i.get_str("description")).bind(3, bytes_of(i, "symptoms_json"));
  s.bind(4, i.get_str("root_cause")).bind(5, i.get_str("resolution")).bind(6, i.get_str("resolved_by"));
  s.bind(7, i.get_str("prevention")).bind(8, ts_of(i, "timestamp"));
  const std::string b = emb_blob(emb);
  s.bind_blob(9, b.data(), b.size()).exec();
}
void MemoryStore::store_config_change(const Json& c) {
  std::lock_guard<std::recursive_mutex> l(lt_.mutex());
  Stmt s(lt_, "INSERT OR REPLACE INTO config_changes VALUES (?1,?2,?3,?4,?5,?6)");
  s.bind(1, id_of(c)).bind(2, c.get_str("file_path")).bind(3, c.get_str("content"));
  s.bind(4, c.get_str("changed_by")).bind(5, c.get_str("reason")).bind(6, ts_of(c, "timestamp")).exec();
}

Json MemoryStore::semantic_search(const std::string& query, const std::vector<std::string>& cols_in, int n,
                                  double min_rel) {
  // hybrid relevance = 0.4 * keyword overlap + 0.6 * cosine(hashed embeddings)  (longterm.rs:186)
  // scored over the whole collection (the reference scored only the N most recent rows)
  const Scorer score(query);
  std::vector<std::string> cols = cols_in;
  if (cols.empty()) cols = {"procedures", "incidents", "config_changes"};
  TopN top(n <= 0 ? 10 : n);
  std::lock_guard<std::recursive_mutex> l(lt_.mutex());
  std::set<std::string> done;
  for (auto& c : cols) {
    const std::string coll = (c == "decisions") ? "procedures" : c;
    if (!done.insert(coll).second) continue;
    if (coll == "procedures") {
      Stmt s(lt_, "SELECT id, name, description, embedding, steps_json FROM procedures ORDER BY last_used DESC LIMIT 5000");
      while (s.step()) {
        const std::string content = s.col_text(1) + ": " + s.col_text(2);
        const double r = score(content, s.col_blob(3));
        if (r < min_rel || !top.wants(r)) {
          top.skip();
          continue;
        }
        top.push(r, Json::object({{"id", s.col_text(0)}, {"content", content},
                                  {"metadata_json", Json::object({{"steps", s.col_text(4)}}).dump()},
                                  {"relevance", r}, {"collection", "procedures"}}));
      }
    } else if (coll == "incidents") {
      Stmt s(lt_, "SELECT id, description, root_cause, resolution, embedding FROM incidents ORDER BY timestamp DESC LIMIT 5000");
      while (s.step()) {
        const std::string content = s.col_text(1) + " | cause: " + s.col_text(2) + " | fix: " + s.col_text(3);
        const double r = score(content, s.col_blob(4));
        if (r < min_rel || !top.wants(r)) {
          top.skip();
          continue;
        }
        top.push(r, Json::object({{"id", s.col_text(0)}, {"content", content}, {"metadata_json", ""},
                                  {"relevance", r}, {"collection", "incidents"}}));
      }
    } else if (coll == "config_changes") {
      Stmt s(lt_, "SELECT id, file_path, reason, changed_by FROM config_changes ORDER BY timestamp DESC LIMIT 5000");
      while (s.step()) {
        const std::string content = s.col_text(1) + ": " + s.col_text(2) + " (by " + s.col_text(3) + ")";
        const double r = score(content, emb_blob(hashed_embedding(content)));
        if (r < min_rel || !top.wants(r)) {
          top.skip();
          continue;
        }
        top.push(r, Json::object({{"id", s.col_text(0)}, {"content", content}, {"metadata_json", ""},
                                  {"relevance", r}, {"collection", "config_changes"}}));
      }
    }
  }
  return top.take();
}

// ---- knowledge
void MemoryStore::add_knowledge(const Json& k) {
  std::lock_guard<std::recursive_mutex> l(kn_.mutex());
  std::string tags;
  for (auto& t : k["tags"].as_arr()) tags += (tags.empty() ? "" : ",") + t.as_str();
  const auto emb = hashed_embedding(k.get_str("title") + " " + k.get_str("content") + " " + tags);
  Stmt s(kn_, "INSERT INTO knowledge VALUES (?1,?2,?3,?4,?5,?6,?7)");
  s.bind(1, id_of(k)).bind(2, k.get_str("title")).bind(3, k.get_str("content")).bind(4, k.get_str("source"));
  s.bind(5, tags).bind(6, now_unix());
  const std::string b = emb_blob(emb);
  s.bind_blob(7, b.data(), b.size()).exec();
}
Json MemoryStore::search_knowledge(const std::string& query, int n, double min_rel) {
  const Scorer score(query);
  TopN top(n <= 0 ? 5 : n);
  std::lock_guard<std::recursive_mutex> l(kn_.mutex());
  Stmt s(kn_, "SELECT id, title, content, source, tags, embedding FROM knowledge LIMIT 20000");
  while (s.step()) {
    const std::string content = s.col_text(1) + ": " + s.col_text(2), tags = s.col_text(4);
    const double r = score(content + " " + tags, s.col_blob(5));
    if (r < min_rel || !top.wants(r)) {
      top.skip();
      continue;
    }
    top.push(r, Json::object({{"id", s.col_text(0)}, {"content", content},
                              {"metadata_json", Json::object({{"source", s.col_text(3)}, {"tags", tags}}).dump()},
                              {"relevance", r}, {"collection", "knowledge"}}));
  }
  return top.take();
}

// ---- context assembly
Json MemoryStore::assemble_context(const std::string& task, int max_tokens, const std::vector<std::string>& tiers_in) {
  const int budget = max_tokens <= 0 ? 4000 : max_tokens;
  std::vector<std::string> tiers = tiers_in;
  if (tiers.empty()) tiers = {"operational", "working", "longterm", "knowledge"};
  std::vector<Json> chunks;
  int total = 0;
  auto add = [&](const char* src, const std::string& content, double rel) -> bool {
    const int t = estimate_tokens(content);
    if (total + t > budget) return false;
    chunks.push_back(Json::object({{"source", src}, {"content", content}, {"relevance", rel}, {"tokens", t}}));
    total += t;
    return true;
  };
  for (auto& tier : tiers) {
    if (total >= budget) break;
    if (tier == "operational") {
      const Json recent = op_.recent(10, "", "");
      for (auto& e : recent.as_arr())
        if (!add("operational", e.get_str("data_json"), 0.8)) break;
    } else if (tier == "working") {
      Json goals = active_goals();
      for (size_t i = 0; i < goals.size() && i < 5; ++i) {
        const Json& g = goals[i];
        if (!add("working", "Goal [" + g.get_str("id") + "]: " + g.get_str("description") + " (status: " +
                                g.get_str("status") + ")",
                 0.7))
          break;
      }
    } else if (tier == "longterm") {
      const Json hits = semantic_search(task, {"decisions", "procedures"}, 5, 0.3);
      for (auto& r : hits.as_arr())
        if (!add("longterm", r.get_str("content"), r.get_num("relevance"))) break;
    } else if (tier == "knowledge") {
      const Json hits = search_knowledge(task, 5, 0.0);
      for (auto& r : hits.as_arr())
        if (!add("knowledge", r.get_str("content"), r.get_num("relevance"))) break;
    }
  }
  std::stable_sort(chunks.begin(), chunks.end(),
                   [](const Json& a, const Json& b) { return a.get_num("relevance") > b.get_num("relevance"); });
  Json arr = Json::array();
  for (auto& c : chunks) arr.push(c);
  return Json::object({{"chunks", arr}, {"total_tokens", total}});
}

// ---- migration
Json MemoryStore::migrate(int64_t max_goal_age_s, int max_patterns, int64_t max_call_age_s) {
  const int64_t now = now_unix();
  int moved = 0, pruned = 0, calls = 0;
  std::vector<Json> done_goals;
  {
    std::lock_guard<std::recursive_mutex> l(work_.mutex());
    Stmt s(work_, "SELECT * FROM goals WHERE status IN ('completed','failed') AND completed_at > 0 AND completed_at < ?1");
    s.bind(1, now - max_goal_age_s);
    while (s.step()) done_goals.push_back(goal_row(s));
  }
  for (auto& g : done_goals) {
    const std::string gid = g.get_str("id");
    Json tasks = tasks_for_goal(gid);
    Json steps = Json::array();
    int64_t dur = 0;
    for (auto& t : tasks.as_arr()) {
      steps.push(Json::object({{"description", t.get_str("description")}, {"agent", t.get_str("agent")},
                               {"status", t.get_str("status")}}));
      dur += t.get_int("duration_ms");
    }
    const bool ok = g.get_str("status") == "completed";
    if (ok) learn_pattern_from_goal(gid);
    store_procedure(Json::object({{"id", "goal-" + gid}, {"name", g.get_str("description").substr(0, 120)},
                                  {"description", g.get_str("description") + " => " + g.get_str("result").substr(0, 400)},
                                  {"steps_json", steps.dump()}, {"success_count", ok ? 1 : 0},
                                  {"fail_count", ok ? 0 : 1},
                                  {"avg_duration_ms", tasks.size() ? dur / (int64_t)tasks.size() : 0},
                                  {"tags", Json::array()}, {"created_at", g.get_int("created_at")}}));
    std::lock_guard<std::recursive_mutex> l(work_.mutex());
    Stmt d1(work_, "DELETE FROM tasks WHERE goal_id = ?1");
    d1.bind(1, gid).exec();
    Stmt d2(work_, "DELETE FROM goals WHERE id = ?1");
    d2.bind(1, gid).exec();
    ++moved;
  }
  {
    std::lock_guard<std::recursive_mutex> l(work_.mutex());
    Stmt c(work_, "SELECT COUNT(*) FROM patterns");
    const int64_t np = c.step() ? c.col_int(0) : 0;
    if (np > max_patterns) {
      Stmt d(work_, "DELETE FROM patterns WHERE id IN (SELECT id FROM patterns ORDER BY success_rate ASC, uses ASC,"
                    " last_used ASC LIMIT ?1)");
      d.bind(1, np - max_patterns).exec();
      pruned = (int)(np - max_patterns);
    }
    Stmt d(work_, "DELETE FROM tool_calls WHERE timestamp < ?1");
    d.bind(1, now - max_call_age_s).exec();
    calls = work_.changes();
  }
  return Json::object({{"goals_migrated", moved}, {"patterns_pruned", pruned}, {"tool_calls_deleted", calls}});
}

Json MemoryStore::stats() {
  auto count = [](Db& db, const char* t) {
    std::lock_guard<std::recursive_mutex> l(db.mutex());
    Stmt s(db, std::string("SELECT COUNT(*) FROM ") + t);
    return s.step() ? s.col_int(0) : (int64_t)0;
  };
  return Json::object({{"events", (int64_t)op_.size()}, {"goals", count(work_, "goals")}, {"tasks", count(work_, "tasks")},
                       {"patterns", count(work_, "patterns")}, {"procedures", count(lt_, "procedures")},
                       {"incidents", count(lt_, "incidents")}, {"knowledge", count(kn_, "knowledge")}});
}

}  // namespace aiosn
