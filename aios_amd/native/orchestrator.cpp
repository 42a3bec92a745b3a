// Orchestrator stores: goal engine, agent router, cluster, discovery, decision log, aggregator,
// cron schedules, event bus, system-prompt assembly.  See orchestrator.h for the reference map.
#include "orchestrator.h"

#include <algorithm>
#include <ctime>

#include "memory.h"

namespace aiosn {

// =============================================================================== GoalEngine
static const std::set<std::string> kActiveGoal = {"pending", "planning", "in_progress", "awaiting_input"};

GoalEngine::GoalEngine(const std::string& db_path) : db_(db_path) {
  db_.exec(
      "CREATE TABLE IF NOT EXISTS goals (id TEXT PRIMARY KEY, description TEXT NOT NULL, priority INTEGER NOT NULL,"
      " source TEXT NOT NULL, status TEXT NOT NULL, created_at INTEGER NOT NULL, updated_at INTEGER NOT NULL,"
      " tags TEXT NOT NULL DEFAULT '[]', metadata_json BLOB NOT NULL DEFAULT X'');"
      "CREATE TABLE IF NOT EXISTS tasks (id TEXT PRIMARY KEY, goal_id TEXT NOT NULL, description TEXT NOT NULL,"
      " assigned_agent TEXT NOT NULL DEFAULT '', status TEXT NOT NULL, intelligence_level TEXT NOT NULL DEFAULT '',"
      " required_tools TEXT NOT NULL DEFAULT '[]', depends_on TEXT NOT NULL DEFAULT '[]', input_json BLOB,"
      " output_json BLOB, created_at INTEGER NOT NULL DEFAULT 0, started_at INTEGER NOT NULL DEFAULT 0,"
      " completed_at INTEGER NOT NULL DEFAULT 0, error TEXT NOT NULL DEFAULT '', seq INTEGER NOT NULL DEFAULT 0);"
      "CREATE TABLE IF NOT EXISTS messages (id TEXT PRIMARY KEY, goal_id TEXT NOT NULL, sender TEXT NOT NULL,"
      " content TEXT NOT NULL, timestamp INTEGER NOT NULL);"
      "CREATE INDEX IF NOT EXISTS idx_tasks_goal ON tasks(goal_id);"
      "CREATE INDEX IF NOT EXISTS idx_messages_goal ON messages(goal_id);");
  // restore state (write-through cache)
  {
    Stmt s(db_, "SELECT id, description, priority, source, status, created_at, updated_at, tags, metadata_json FROM goals");
    while (s.step()) {
      Json tags;
      if (!Json::try_parse(s.col_text(7), tags)) tags = Json::array();
      Json g = Json::object({{"id", s.col_text(0)}, {"description", s.col_text(1)}, {"priority", s.col_int(2)},
                             {"source", s.col_text(3)}, {"status", s.col_text(4)}, {"created_at", s.col_int(5)},
                             {"updated_at", s.col_int(6)}, {"tags", tags}, {"metadata_json", s.col_blob(8)}});
      goals_[g.get_str("id")] = g;
    }
  }
  {
    Stmt s(db_, "SELECT id, goal_id, description, assigned_agent, status, intelligence_level, required_tools, depends_on,"
                " input_json, output_json, created_at, started_at, completed_at, error FROM tasks ORDER BY seq ASC");
    while (s.step()) {
      Json rt, dep;
      if (!Json::try_parse(s.col_text(6), rt)) rt = Json::array();
      if (!Json::try_parse(s.col_text(7), dep)) dep = Json::array();
      Json t = Json::object({{"id", s.col_text(0)}, {"goal_id", s.col_text(1)}, {"description", s.col_text(2)},
                             {"assigned_agent", s.col_text(3)}, {"status", s.col_text(4)},
                             {"intelligence_level", s.col_text(5)}, {"required_tools", rt}, {"depends_on", dep},
                             {"input_json", s.col_blob(8)}, {"output_json", s.col_blob(9)}, {"created_at", s.col_int(10)},
                             {"started_at", s.col_int(11)}, {"completed_at", s.col_int(12)}, {"error", s.col_text(13)}});
      task_order_.push_back(t.get_str("id"));
      tasks_[t.get_str("id")] = t;
    }
  }
}

void GoalEngine::persist_goal(const Json& g) {
  Stmt s(db_, "INSERT OR REPLACE INTO goals VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9)");
  const std::string meta = g.get_str("metadata_json");
  s.bind(1, g.get_str("id")).bind(2, g.get_str("description")).bind(3, g.get_int("priority"));
  s.bind(4, g.get_str("source")).bind(5, g.get_str("status")).bind(6, g.get_int("created_at"));
  s.bind(7, g.get_int("updated_at")).bind(8, g["tags"].dump()).bind_blob(9, meta.data(), meta.size()).exec();
}
void GoalEngine::persist_task(const Json& t) {
  Stmt s(db_, "INSERT OR REPLACE INTO tasks VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9,?10,?11,?12,?13,?14,?15)");
  const std::string in = t.get_str("input_json"), out = t.get_str("output_json");
  auto it = std::find(task_order_.begin(), task_order_.end(), t.get_str("id"));
  s.bind(1, t.get_str("id")).bind(2, t.get_str("goal_id")).bind(3, t.get_str("description"));
  s.bind(4, t.get_str("assigned_agent")).bind(5, t.get_str("status")).bind(6, t.get_str("intelligence_level"));
  s.bind(7, t["required_tools"].dump()).bind(8, t["depends_on"].dump()).bind_blob(9, in.data(), in.size());
  s.bind_blob(10, out.data(), out.size()).bind(11, t.get_int("created_at")).bind(12, t.get_int("started_at"));
  s.bind(13, t.get_int("completed_at")).bind(14, t.get_str("error")).bind(15, (int64_t)(it - task_order_.begin())).exec();
}

Json GoalEngine::submit(const std::string& description, int priority, const std::string& source, const Json& tags,
                        const std::string& metadata_json) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  const int64_t now = now_unix();
  Json g = Json::object({{"id", uuid4()}, {"description", description}, {"priority", priority ? priority : 5},
                         {"source", source.empty() ? "user" : source}, {"status", "pending"}, {"created_at", now},
                         {"updated_at", now}, {"tags", tags.is_arr() ? tags : Json::array()},
                         {"metadata_json", metadata_json}});
  goals_[g.get_str("id")] = g;
  persist_goal(g);
  return g;
}
Json GoalEngine::goal(const std::string& id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto it = goals_.find(id);
  return it == goals_.end() ? Json::object() : it->second;
}
Json GoalEngine::list(const std::string& status, int limit, int offset, int& total) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  std::vector<const Json*> v;
  for (auto& kv : goals_)
    if (status.empty() || kv.second.get_str("status") == status) v.push_back(&kv.second);
  // priority ascending, newest first (goal_engine.rs:328-362)
  std::sort(v.begin(), v.end(), [](const Json* a, const Json* b) {
    if (a->get_int("priority") != b->get_int("priority")) return a->get_int("priority") < b->get_int("priority");
    return a->get_int("created_at") > b->get_int("created_at");
  });
  total = (int)v.size();
  Json out = Json::array();
  const int lim = limit > 0 ? limit : 50;
  for (int i = std::max(0, offset); i < (int)v.size() && (int)out.size() < lim; ++i) out.push(*v[i]);
  return out;
}
bool GoalEngine::cancel(const std::string& id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto it = goals_.find(id);
  if (it == goals_.end()) return false;
  const std::string st = it->second.get_str("status");
  if (st == "completed" || st == "failed" || st == "cancelled") return false;
  it->second.set("status", "cancelled");
  it->second.set("updated_at", now_unix());
  persist_goal(it->second);
  for (auto& kv : tasks_) {
    if (kv.second.get_str("goal_id") != id) continue;
    const std::string ts = kv.second.get_str("status");
    if (ts != "completed" && ts != "failed") {
      kv.second.set("status", "cancelled");
      persist_task(kv.second);
    }
  }
  return true;
}
void GoalEngine::set_goal_status(const std::string& id, const std::string& status) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto it = goals_.find(id);
  if (it == goals_.end()) return;
  it->second.set("status", status);
  it->second.set("updated_at", now_unix());
  persist_goal(it->second);
}
void GoalEngine::set_goal_metadata(const std::string& id, const std::string& key, const Json& value) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto it = goals_.find(id);
  if (it == goals_.end()) return;
  Json meta;
  if (!Json::try_parse(it->second.get_str("metadata_json"), meta) || !meta.is_obj()) meta = Json::object();
  meta.set(key, value);
  it->second.set("metadata_json", meta.dump());
  persist_goal(it->second);
}
void GoalEngine::add_tasks(const std::string& goal_id, const Json& tasks) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  for (auto& t : tasks.as_arr()) {
    Json tt = t;
    tt.set("goal_id", goal_id);
    if (tt.get_str("id").empty()) tt.set("id", uuid4());
    if (!tasks_.count(tt.get_str("id"))) task_order_.push_back(tt.get_str("id"));
    tasks_[tt.get_str("id")] = tt;
    persist_task(tt);
  }
  auto it = goals_.find(goal_id);
  if (it != goals_.end() && it->second.get_str("status") == "pending") {
    it->second.set("status", "in_progress");
    it->second.set("updated_at", now_unix());
    persist_goal(it->second);
  }
}
Json GoalEngine::task(const std::string& id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto it = tasks_.find(id);
  return it == tasks_.end() ? Json::object() : it->second;
}
Json GoalEngine::tasks_for_goal(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  Json out = Json::array();
  for (auto& id : task_order_) {
    auto it = tasks_.find(id);
    if (it != tasks_.end() && it->second.get_str("goal_id") == goal_id) out.push(it->second);
  }
  return out;
}
void GoalEngine::update_task(const Json& t) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  const std::string id = t.get_str("id");
  auto it = tasks_.find(id);
  if (it == tasks_.end()) {
    task_order_.push_back(id);
    tasks_[id] = t;
  } else {
    for (auto& kv : t.as_obj()) it->second.set(kv.first, kv.second);
  }
  persist_task(tasks_[id]);
}
Json GoalEngine::next_tasks(int max) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  Json out = Json::array();
  for (auto& id : task_order_) {
    if ((int)out.size() >= max) break;
    auto& t = tasks_[id];
    if (t.get_str("status") != "pending") continue;
    auto g = goals_.find(t.get_str("goal_id"));
    if (g != goals_.end() && (g->second.get_str("status") == "cancelled" || g->second.get_str("status") == "failed"))
      continue;
    bool ready = true;
    for (auto& d : t["depends_on"].as_arr()) {
      auto dt = tasks_.find(d.as_str());
      if (dt != tasks_.end() && dt->second.get_str("status") != "completed") {
        ready = false;
        break;
      }
    }
    if (ready) out.push(t);
  }
  return out;
}
double GoalEngine::progress(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  int n = 0, done = 0;
  for (auto& kv : tasks_)
    if (kv.second.get_str("goal_id") == goal_id) {
      ++n;
      if (kv.second.get_str("status") == "completed") ++done;
    }
  auto g = goals_.find(goal_id);
  if (n == 0) return (g != goals_.end() && g->second.get_str("status") == "completed") ? 100.0 : 0.0;
  return 100.0 * done / n;
}
std::string GoalEngine::phase(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto g = goals_.find(goal_id);
  if (g == goals_.end()) return "";
  const std::string st = g->second.get_str("status");
  if (st != "in_progress") return st;
  for (auto& id : task_order_) {
    auto& t = tasks_[id];
    if (t.get_str("goal_id") == goal_id && t.get_str("status") != "completed") return "executing: " + t.get_str("description");
  }
  return "finalizing";
}
std::string GoalEngine::check_completion(const std::string& goal_id) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  auto g = goals_.find(goal_id);
  if (g == goals_.end()) return "";
  const std::string st = g->second.get_str("status");
  if (st == "completed" || st == "failed" || st == "cancelled") return "";
  int n = 0, done = 0, failed = 0;
  for (auto& kv : tasks_) {
    if (kv.second.get_str("goal_id") != goal_id) continue;
    ++n;
    const std::string ts = kv.second.get_str("status");
    if (ts == "completed") ++done;
    else if (ts == "failed") ++failed;
  }
  if (n == 0) return "";
  std::string ns;
  if (failed > 0) ns = "failed";
  else if (done == n) ns = "completed";
  if (!ns.empty()) {
    g->second.set("status", ns);
    g->second.set("updated_at", now_unix());
    persist_goal(g->second);
  }
  return ns;
}
void GoalEngine::add_message(const std::string& goal_id, const std::string& sender, const std::string& content) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  Stmt s(db_, "INSERT INTO messages VALUES (?1,?2,?3,?4,?5)");
  s.bind(1, uuid4()).bind(2, goal_id).bind(3, sender).bind(4, content).bind(5, now_ms()).exec();
}
Json GoalEngine::messages(const std::string& goal_id, int limit) {
  std::lock_guard<std::recursive_mutex> l(mu_);
  Stmt s(db_, "SELECT sender, content, timestamp FROM (SELECT * FROM messages WHERE goal_id = ?1 ORDER BY timestamp DESC"
              " LIMIT ?2) ORDER BY timestamp ASC");
  s.bind(1, goal_id).bind(2, (int64_t)(limit > 0 ? limit : 50));
  Json out = Json::array();
  while (s.step())
    out.push(Json::object({{"sender", s.col_text(0)}, {"content", s.col_text(1)}, {"timestamp", s.col_int(2)}}));
  return out;
}
int GoalEngine::resume_in_progress() {
  std::lock_guard<std::recursive_mutex> l(mu_);
  int n = 0;
  for (auto& kv : tasks_) {
    const std::string st = kv.second.get_str("status");
    if (st == "in_progress" || st == "assigned") {
      kv.second.set("status", "pending");
      kv.second.set("assigned_agent", "");
      persist_task(kv.second);
      ++n;
    }
  }
  return n;
}
Json GoalEngine::counts() {
  std::lock_guard<std::recursive_mutex> l(mu_);
  int active = 0, pending_t = 0, inprog_t = 0, awaiting = 0;
  for (auto& kv : goals_)
    if (kActiveGoal.count(kv.second.get_str("status"))) ++active;
  for (auto& kv : tasks_) {
    const std::string st = kv.second.get_str("status");
    if (st == "pending") ++pending_t;
    else if (st == "in_progress" || st == "assigned") ++inprog_t;
    else if (st == "awaiting_input") ++awaiting;
  }
  return Json::object({{"active_goals", active}, {"pending_tasks", pending_t}, {"in_progress_tasks", inprog_t},
                       {"awaiting_input_tasks", awaiting}, {"total_goals", (int64_t)goals_.size()},
                       {"total_tasks", (int64_t)tasks_.size()}});
}
Json GoalEngine::pending_goals_without_tasks() {
  std::lock_guard<std::recursive_mutex> l(mu_);
  std::set<std::string> with;
  for (auto& kv : tasks_) with.insert(kv.second.get_str("goal_id"));
  std::vector<const Json*> v;
  for (auto& kv : goals_)
    if (kv.second.get_str("status") == "pending" && !with.count(kv.first)) v.push_back(&kv.second);
  std::sort(v.begin(), v.end(), [](const Json* a, const Json* b) {
    if (a->get_int("priority") != b->get_int("priority")) return a->get_int("priority") < b->get_int("priority");
    return a->get_int("created_at") < b->get_int("created_at");
  });
  Json out = Json::array();
  for (auto* g : v) out.push(*g);
  return out;
}

// =============================================================================== AgentRouter
void AgentRouter::register_agent(const Json& reg) {
  std::lock_guard<std::mutex> l(mu_);
  Agent& a = agents_[reg.get_str("agent_id")];
  a.reg = reg;
  if (!a.reg.get_int("registered_at")) a.reg.set("registered_at", now_unix());
  a.status = "idle";
  a.last_hb = now_unix();
}
bool AgentRouter::unregister(const std::string& id) {
  std::lock_guard<std::mutex> l(mu_);
  return agents_.erase(id) > 0;
}
bool AgentRouter::heartbeat(const std::string& id, const std::string& status, const std::string& task_id) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = agents_.find(id);
  if (it == agents_.end()) return false;
  it->second.last_hb = now_unix();
  if (!status.empty()) it->second.status = status;
  if (!task_id.empty()) it->second.task = task_id;
  return true;
}
bool AgentRouter::healthy(const Agent& a) const { return now_unix() - a.last_hb <= timeout_; }
Json AgentRouter::list() {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto& kv : agents_) {
    Json r = kv.second.reg;
    r.set("status", healthy(kv.second) ? kv.second.status : std::string("unresponsive"));
    out.push(r);
  }
  return out;
}
std::string AgentRouter::route(const Json& task) {
  // healthy + idle + namespace / capability-prefix match, then a busy-but-capable agent; prefer
  // idle, then the most completed tasks (agent_router.rs:73-141)
  std::lock_guard<std::mutex> l(mu_);
  std::vector<std::string> tools;
  for (auto& t : task["required_tools"].as_arr()) tools.push_back(t.as_str());
  auto capable = [&](const Agent& a) {
    if (tools.empty()) return false;
    for (auto& t : tools) {
      bool ok = false;
      for (auto& ns : a.reg["tool_namespaces"].as_arr())
        if (ns.as_str() == t) ok = true;
      for (auto& c : a.reg["capabilities"].as_arr())
        if (starts_with(c.as_str(), t + ".") || c.as_str() == t) ok = true;
      if (!ok) return false;
    }
    return true;
  };
  std::string best;
  int best_score = -1;
  for (auto& kv : agents_) {
    const Agent& a = kv.second;
    if (!healthy(a) || !capable(a)) continue;
    const bool idle = a.status == "idle" && a.task.empty();
    const int score = (idle ? 1000000 : 0) + a.completed;
    if (score > best_score) {
      best_score = score;
      best = kv.first;
    }
  }
  return best;
}
void AgentRouter::assign(const std::string& agent, const std::string& task_id) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = agents_.find(agent);
  if (it == agents_.end()) return;
  it->second.task = task_id;
  it->second.status = "busy";
}
void AgentRouter::task_completed(const std::string& agent, bool success) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = agents_.find(agent);
  if (it == agents_.end()) return;
  it->second.task.clear();
  it->second.status = "idle";
  (success ? it->second.completed : it->second.failed)++;
}
Json AgentRouter::dead_agents() {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto& kv : agents_)
    if (!healthy(kv.second)) out.push(Json::object({{"agent_id", kv.first}, {"task_id", kv.second.task}}));
  return out;
}
int AgentRouter::healthy_count() {
  std::lock_guard<std::mutex> l(mu_);
  int n = 0;
  for (auto& kv : agents_) n += healthy(kv.second);
  return n;
}

// =============================================================================== cluster
void ClusterManager::register_node(const Json& n) {
  std::lock_guard<std::mutex> l(mu_);
  Json node = n;
  if (!node.has("cpu_usage")) node.set("cpu_usage", 0.0);
  if (!node.has("memory_usage")) node.set("memory_usage", 0.0);
  if (!node.has("active_tasks")) node.set("active_tasks", 0);
  if (node.get_int("max_tasks") <= 0) node.set("max_tasks", 10);
  nodes_[n.get_str("node_id")] = node;
  last_[n.get_str("node_id")] = now_unix();
}
bool ClusterManager::heartbeat(const std::string& node, double cpu, double mem, int active) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return false;
  it->second.set("cpu_usage", cpu);
  it->second.set("memory_usage", mem);
  it->second.set("active_tasks", active);
  last_[node] = now_unix();
  return true;
}
Json ClusterManager::list(bool include_dead) {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  const int64_t now = now_unix();
  for (auto& kv : nodes_) {
    const bool ok = now - last_[kv.first] <= timeout_;
    if (!ok && !include_dead) continue;
    Json n = kv.second;
    n.set("healthy", ok);
    out.push(n);
  }
  return out;
}
std::string ClusterManager::route_least_loaded() {
  // load = cpu + active/max*100 (cluster.rs:110-128)
  std::lock_guard<std::mutex> l(mu_);
  std::string best;
  double best_load = 1e18;
  const int64_t now = now_unix();
  for (auto& kv : nodes_) {
    if (now - last_[kv.first] > timeout_) continue;
    const double mx = (double)std::max<int64_t>(1, kv.second.get_int("max_tasks"));
    if (kv.second.get_int("active_tasks") >= (int64_t)mx) continue;
    const double load = kv.second.get_num("cpu_usage") + (double)kv.second.get_int("active_tasks") / mx * 100.0;
    if (load < best_load) {
      best_load = load;
      best = kv.first;
    }
  }
  return best;
}
int ClusterManager::prune() {
  std::lock_guard<std::mutex> l(mu_);
  int n = 0;
  const int64_t now = now_unix();
  for (auto it = nodes_.begin(); it != nodes_.end();) {
    if (now - last_[it->first] > timeout_ * 4) {
      last_.erase(it->first);
      it = nodes_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  return n;
}

// =============================================================================== discovery
Discovery::Discovery(int ttl_s) : ttl_(ttl_s) {
  // the six default services (discovery.rs:58-82)
  register_service("orchestrator", "127.0.0.1", 50051, "grpc");
  register_service("tools", "127.0.0.1", 50052, "grpc");
  register_service("memory", "127.0.0.1", 50053, "grpc");
  register_service("api-gateway", "127.0.0.1", 50054, "grpc");
  register_service("runtime", "127.0.0.1", 50055, "grpc");
  register_service("management", "127.0.0.1", 9090, "http");
}
void Discovery::register_service(const std::string& name, const std::string& address, int port,
                                 const std::string& proto) {
  std::lock_guard<std::mutex> l(mu_);
  svc_[name] = Json::object({{"name", name}, {"address", address}, {"port", port}, {"protocol", proto},
                             {"status", "registered"}, {"registered_at", now_unix()}});
  seen_[name] = now_unix();
}
bool Discovery::heartbeat(const std::string& name) {
  std::lock_guard<std::mutex> l(mu_);
  if (!svc_.count(name)) return false;
  seen_[name] = now_unix();
  return true;
}
Json Discovery::lookup(const std::string& name) {
  std::lock_guard<std::mutex> l(mu_);
  auto it = svc_.find(name);
  if (it == svc_.end()) return Json::object();
  return it->second;
}
Json Discovery::list() {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto& kv : svc_) {
    Json s = kv.second;
    s.set("status", now_unix() - seen_[kv.first] <= ttl_ ? "healthy" : "stale");
    out.push(s);
  }
  return out;
}
int Discovery::prune() {
  // defaults are static and never pruned; dynamically registered services expire after 4 TTLs
  std::lock_guard<std::mutex> l(mu_);
  static const std::set<std::string> defaults = {"orchestrator", "tools", "memory", "api-gateway", "runtime", "management"};
  int n = 0;
  for (auto it = svc_.begin(); it != svc_.end();) {
    if (!defaults.count(it->first) && now_unix() - seen_[it->first] > ttl_ * 4) {
      seen_.erase(it->first);
      it = svc_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  return n;
}

// =============================================================================== decisions
std::string DecisionLog::log(const std::string& context, const Json& options, const std::string& chosen,
                             const std::string& reasoning, const std::string& level, const std::string& model) {
  std::lock_guard<std::mutex> l(mu_);
  const std::string id = uuid4();
  ring_.push_back(Json::object({{"id", id}, {"context", context}, {"options", options}, {"chosen", chosen},
                                {"reasoning", reasoning}, {"intelligence_level", level}, {"model_used", model},
                                {"outcome", ""}, {"timestamp", now_unix()}}));
  while (ring_.size() > cap_) ring_.pop_front();
  return id;
}
bool DecisionLog::update_outcome(const std::string& id, const std::string& outcome) {
  std::lock_guard<std::mutex> l(mu_);
  for (auto it = ring_.rbegin(); it != ring_.rend(); ++it)
    if (it->get_str("id") == id) {
      it->set("outcome", outcome);
      return true;
    }
  return false;
}
double DecisionLog::success_rate(const std::string& ctx) {
  std::lock_guard<std::mutex> l(mu_);
  int n = 0, ok = 0;
  for (auto& d : ring_) {
    if (!ctx.empty() && !contains(d.get_str("context"), ctx)) continue;
    const std::string o = d.get_str("outcome");
    if (o.empty()) continue;
    ++n;
    if (o == "success" || o == "completed") ++ok;
  }
  return n ? (double)ok / n : 0.0;
}
Json DecisionLog::recent(int n) {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto it = ring_.rbegin(); it != ring_.rend() && (int)out.size() < n; ++it) out.push(*it);
  return out;
}
size_t DecisionLog::size() {
  std::lock_guard<std::mutex> l(mu_);
  return ring_.size();
}

// =============================================================================== aggregator
void ResultAggregator::record(const std::string& goal_id, const Json& result) {
  std::lock_guard<std::mutex> l(mu_);
  by_goal_[goal_id].push_back(result);
}
Json ResultAggregator::results(const std::string& goal_id) {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto& r : by_goal_[goal_id]) out.push(r);
  return out;
}
Json ResultAggregator::summary(const std::string& goal_id) {
  std::lock_guard<std::mutex> l(mu_);
  auto& v = by_goal_[goal_id];
  int ok = 0;
  int64_t tokens = 0, dur = 0;
  std::set<std::string> models;
  for (auto& r : v) {
    ok += r.get_bool("success");
    tokens += r.get_int("tokens_used");
    dur += r.get_int("duration_ms");
    if (!r.get_str("model_used").empty()) models.insert(r.get_str("model_used"));
  }
  Json m = Json::array();
  for (auto& x : models) m.push(x);
  return Json::object({{"goal_id", goal_id}, {"total_tasks", (int64_t)v.size()}, {"successful", ok},
                       {"failed", (int64_t)v.size() - ok}, {"total_tokens", tokens}, {"total_duration_ms", dur},
                       {"models_used", m}});
}

// =============================================================================== cron
namespace {
bool cron_field(const std::string& f, int value, int lo, int hi) {
  for (auto& part : split(f, ',')) {
    const std::string p = trim(part);
    if (p == "*") return true;
    if (starts_with(p, "*/")) {
      const int step = std::atoi(p.c_str() + 2);
      if (step > 0 && (value - lo) % step == 0) return true;
      continue;
    }
    const auto dash = p.find('-');
    if (dash != std::string::npos) {
      const int a = std::atoi(p.substr(0, dash).c_str()), b = std::atoi(p.substr(dash + 1).c_str());
      if (value >= a && value <= b) return true;
      continue;
    }
    if (!p.empty() && std::isdigit((unsigned char)p[0]) && std::atoi(p.c_str()) == value) return true;
  }
  (void)hi;
  return false;
}
}  // namespace

bool cron_valid(const std::string& expr) {
  auto f = split_ws(expr);
  if (f.size() != 5) return false;
  for (auto& x : f)
    for (char c : x)
      if (!(std::isdigit((unsigned char)c) || c == '*' || c == '/' || c == ',' || c == '-')) return false;
  return true;
}

bool cron_matches(const std::string& expr, int64_t t) {
  // minute hour day-of-month month day-of-week (scheduler.rs:187-207; UTC)
  auto f = split_ws(expr);
  if (f.size() != 5) return false;
  std::time_t tt = (std::time_t)t;
  std::tm tm{};
  gmtime_r(&tt, &tm);
  return cron_field(f[0], tm.tm_min, 0, 59) && cron_field(f[1], tm.tm_hour, 0, 23) &&
         cron_field(f[2], tm.tm_mday, 1, 31) && cron_field(f[3], tm.tm_mon + 1, 1, 12) &&
         cron_field(f[4], tm.tm_wday, 0, 6);
}

ScheduleStore::ScheduleStore(const std::string& db_path) : db_(db_path) {
  db_.exec("CREATE TABLE IF NOT EXISTS scheduled_goals (id TEXT PRIMARY KEY, cron_expr TEXT NOT NULL,"
           " goal_template TEXT NOT NULL, priority INTEGER NOT NULL, enabled INTEGER NOT NULL DEFAULT 1,"
           " last_run INTEGER NOT NULL DEFAULT 0)");
}
std::string ScheduleStore::create(const std::string& cron, const std::string& tmpl, int priority) {
  if (!cron_valid(cron)) throw std::runtime_error("invalid cron expression: " + cron);
  std::lock_guard<std::mutex> l(mu_);
  const std::string id = uuid4();
  Stmt s(db_, "INSERT INTO scheduled_goals VALUES (?1,?2,?3,?4,1,0)");
  s.bind(1, id).bind(2, cron).bind(3, tmpl).bind(4, (int64_t)(priority ? priority : 5)).exec();
  return id;
}
Json ScheduleStore::list() {
  std::lock_guard<std::mutex> l(mu_);
  Stmt s(db_, "SELECT id, cron_expr, goal_template, priority, enabled, last_run FROM scheduled_goals");
  Json out = Json::array();
  while (s.step())
    out.push(Json::object({{"id", s.col_text(0)}, {"cron_expr", s.col_text(1)}, {"goal_template", s.col_text(2)},
                           {"priority", s.col_int(3)}, {"enabled", s.col_int(4) != 0}, {"last_run", s.col_int(5)}}));
  return out;
}
bool ScheduleStore::remove(const std::string& id) {
  std::lock_guard<std::mutex> l(mu_);
  Stmt s(db_, "DELETE FROM scheduled_goals WHERE id = ?1");
  s.bind(1, id).exec();
  return db_.changes() > 0;
}
Json ScheduleStore::due(int64_t now) {
  Json all = list();
  Json out = Json::array();
  const int64_t minute = now / 60;
  std::lock_guard<std::mutex> l(mu_);
  for (auto& e : all.as_arr()) {
    if (!e.get_bool("enabled") || !cron_matches(e.get_str("cron_expr"), now)) continue;
    if (e.get_int("last_run") / 60 == minute) continue;  // at most once per minute
    Stmt s(db_, "UPDATE scheduled_goals SET last_run = ?2 WHERE id = ?1");
    s.bind(1, e.get_str("id")).bind(2, now).exec();
    out.push(e);
  }
  return out;
}

// =============================================================================== event bus
int EventBus::sev(const std::string& s) {
  const std::string l = lower(s);
  if (l == "critical") return 4;
  if (l == "error" || l == "high") return 3;
  if (l == "warning" || l == "warn" || l == "medium") return 2;
  if (l == "info" || l == "low") return 1;
  return 0;
}
std::string EventBus::subscribe(const std::string& pattern, const std::string& min_sev, const std::string& tmpl,
                                int priority) {
  std::lock_guard<std::mutex> l(mu_);
  const std::string id = uuid4();
  subs_.push_back(Json::object({{"id", id}, {"pattern", pattern}, {"min_severity", min_sev}, {"goal_template", tmpl},
                                {"priority", priority}}));
  return id;
}
bool EventBus::unsubscribe(const std::string& id) {
  std::lock_guard<std::mutex> l(mu_);
  const size_t n = subs_.size();
  subs_.erase(std::remove_if(subs_.begin(), subs_.end(), [&](const Json& s) { return s.get_str("id") == id; }),
              subs_.end());
  return subs_.size() != n;
}
Json EventBus::publish(const Json& ev) {
  std::lock_guard<std::mutex> l(mu_);
  Json e = ev;
  if (!e.get_int("timestamp")) e.set("timestamp", now_unix());
  events_.push_back(e);
  while (events_.size() > 100) events_.pop_front();
  Json goals = Json::array();
  const std::string type = ev.get_str("event_type", ev.get_str("category"));
  for (auto& s : subs_) {
    const std::string pat = s.get_str("pattern");
    bool match = pat == "*" || pat == type || (ends_with(pat, "*") && starts_with(type, pat.substr(0, pat.size() - 1)));
    if (!match || sev(ev.get_str("severity", "info")) < sev(s.get_str("min_severity", "info"))) continue;
    std::string d = s.get_str("goal_template");
    for (auto& kv : std::vector<std::pair<std::string, std::string>>{{"{event_type}", type},
                                                                      {"{source}", ev.get_str("source")},
                                                                      {"{message}", ev.get_str("message")}}) {
      size_t p;
      while ((p = d.find(kv.first)) != std::string::npos) d.replace(p, kv.first.size(), kv.second);
    }
    goals.push(Json::object({{"description", d}, {"priority", s.get_int("priority", 3)},
                             {"subscription_id", s.get_str("id")}}));
  }
  return goals;
}
Json EventBus::recent(int n) {
  std::lock_guard<std::mutex> l(mu_);
  Json out = Json::array();
  for (auto it = events_.rbegin(); it != events_.rend() && (int)out.size() < n; ++it) out.push(*it);
  return out;
}

// =============================================================================== context
std::string build_system_prompt(const std::string& task, const std::string& level, const Json& tools,
                                const Json& patterns, int max_tokens) {
  // context.rs:96-117: task, level, tools, JSON format hint (steps / tools_needed / reasoning);
  // known patterns packed under the remaining budget at 4 chars/token
  std::string p = "You are aiOS, an autonomous AI operating system agent.\nTask: " + task +
                  "\nIntelligence level: " + level + "\n";
  if (tools.size()) {
    p += "Available tools:";
    for (auto& t : tools.as_arr()) p += " " + (t.is_str() ? t.as_str() : t.get_str("name"));
    p += "\n";
  }
  p += "Respond in JSON with fields: \"steps\" (array of {tool, input}), \"tools_needed\" (array of tool names), "
       "\"reasoning\" (string).\n";
  int used = estimate_tokens(p);
  const int budget = max_tokens > 0 ? max_tokens : 2048;
  if (patterns.size()) {
    std::string block = "Known patterns:\n";
    for (auto& pt : patterns.as_arr()) {
      const std::string line = "- when \"" + pt.get_str("trigger") + "\": " + pt.get_str("action") + "\n";
      if (used + estimate_tokens(block + line) > budget) break;
      block += line;
    }
    if (block.size() > 16) p += block;
  }
  return p;
}

}  // namespace aiosn
