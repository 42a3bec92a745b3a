// Orchestrator / control-plane core (MI355X build of the reference's `agent-core/src`).
// The gRPC service and the asyncio autonomy loop (aios_amd/services/orchestrator.py) drive these
// native pieces:
//   GoalEngine      goal lifecycle + per-goal tasks + conversation, write-through SQLite (WAL),
//                   resume of in-progress work after restart          (goal_engine.rs)
//   planner::*      complexity classification, heuristic / AI-response decomposition, tool
//                   namespace inference                                 (task_planner.rs)
//   llm::*          <think> stripping, JSON extraction, tool-call parsing with fallbacks,
//                   clarification parsing, reactive-tier heuristic executor, summaries (autonomy.rs)
//   AgentRouter     registry + heartbeat liveness + capability routing   (agent_router.rs)
//   ClusterManager  multi-node registry, least-loaded routing            (cluster.rs)
//   Discovery       static service registry with TTL                     (discovery.rs)
//   DecisionLog     ring of 10,000 decisions, success rate by context    (decision_logger.rs)
//   ResultAggregator per-goal results summary                            (result_aggregator.rs)
//   ScheduleStore   5-field cron subset persisted in SQLite              (scheduler.rs)
//   EventBus        pattern/severity subscriptions -> goal templates     (event_bus.rs)
//   build_system_prompt  task context under a 4-chars/token budget       (context.rs)
#pragma once
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "json.h"
#include "util.h"

namespace aiosn {

namespace planner {
std::string classify(const std::string& description);           // reactive|operational|tactical|strategic
std::vector<std::string> infer_tools(const std::string& description);
std::vector<std::pair<std::string, std::vector<std::string>>> analyze_steps(const std::string& description);
std::string extract_service_name(const std::string& desc_lower);
// -> tasks (Json array of common.Task dicts), linear depends_on chain, step 0 operational
Json decompose(const std::string& goal_id, const std::string& description, const std::string& level);
Json parse_ai_decomposition(const std::string& text, const std::string& goal_id, const std::string& level);
std::string ai_decomposition_prompt(const std::string& description);
extern const char* kDecomposeSystemPrompt;
}  // namespace planner

namespace llm {
std::string strip_think(const std::string& text);
bool extract_json(const std::string& text, Json& out);
Json parse_tool_calls(const std::string& text);                  // [{tool, input}]
Json tools_from_natural_language(const std::string& text);
bool parse_clarification(const std::string& text, std::string& questions);
Json heuristic_calls(const Json& task);                          // [] when no heuristic applies
bool explicit_tool_call(const std::string& desc, Json& call);
std::string json_to_readable(const Json& v, int depth = 0);
std::string summarize_tool_output(const std::string& tool, const Json& output, size_t max_chars = 1000);
bool is_done_signal(const std::string& text);                    // {"done": true}
}  // namespace llm

class GoalEngine {
 public:
  explicit GoalEngine(const std::string& db_path);  // ":memory:" for tests
  Json submit(const std::string& description, int priority, const std::string& source, const Json& tags,
              const std::string& metadata_json);
  Json goal(const std::string& id);  // {} if missing
  Json list(const std::string& status_filter, int limit, int offset, int& total);
  bool cancel(const std::string& id);
  void set_goal_status(const std::string& id, const std::string& status);
  void set_goal_metadata(const std::string& id, const std::string& key, const Json& value);
  void add_tasks(const std::string& goal_id, const Json& tasks);
  Json task(const std::string& id);
  Json tasks_for_goal(const std::string& goal_id);
  void update_task(const Json& task);
  Json next_tasks(int max);                       // pending tasks with all dependencies completed
  double progress(const std::string& goal_id);
  std::string phase(const std::string& goal_id);
  // goal completion: every task completed -> completed; a failed task -> failed.  Returns new status or ""
  std::string check_completion(const std::string& goal_id);
  void add_message(const std::string& goal_id, const std::string& sender, const std::string& content);
  Json messages(const std::string& goal_id, int limit);
  int resume_in_progress();                       // in_progress/assigned tasks -> pending (restart)
  Json counts();                                  // {active_goals, pending_tasks, ...}
  Json pending_goals_without_tasks();

 private:
  void persist_goal(const Json& g);
  void persist_task(const Json& t);
  std::recursive_mutex mu_;
  Db db_;
  std::map<std::string, Json> goals_;
  std::map<std::string, Json> tasks_;
  std::vector<std::string> task_order_;
};

class AgentRouter {
 public:
  explicit AgentRouter(int heartbeat_timeout_s = 15) : timeout_(heartbeat_timeout_s) {}
  void register_agent(const Json& reg);
  bool unregister(const std::string& id);
  bool heartbeat(const std::string& id, const std::string& status, const std::string& task_id);
  Json list();
  std::string route(const Json& task);           // "" if no agent can take it
  void assign(const std::string& agent, const std::string& task_id);
  void task_completed(const std::string& agent, bool success);
  Json dead_agents();                            // [{agent_id, task_id}] past the heartbeat timeout
  int healthy_count();

 private:
  struct Agent {
    Json reg;
    std::string status = "idle", task;
    int64_t last_hb = 0;
    int completed = 0, failed = 0;
  };
  bool healthy(const Agent& a) const;
  std::mutex mu_;
  std::map<std::string, Agent> agents_;
  int timeout_;
};

class ClusterManager {
 public:
  explicit ClusterManager(int timeout_s = 30) : timeout_(timeout_s) {}
  void register_node(const Json& n);
  bool heartbeat(const std::string& node, double cpu, double mem, int active);
  Json list(bool include_dead);
  std::string route_least_loaded();
  int prune();

 private:
  std::mutex mu_;
  std::map<std::string, Json> nodes_;
  std::map<std::string, int64_t> last_;
  int timeout_;
};

class Discovery {
 public:
  explicit Discovery(int ttl_s = 30);
  void register_service(const std::string& name, const std::string& address, int port, const std::string& proto);
  bool heartbeat(const std::string& name);
  Json lookup(const std::string& name);  // {} if missing / expired
  Json list();
  int prune();

 private:
  std::mutex mu_;
  std::map<std::string, Json> svc_;
  std::map<std::string, int64_t> seen_;
  int ttl_;
};

class DecisionLog {
 public:
  explicit DecisionLog(size_t cap = 10000) : cap_(cap) {}
  std::string log(const std::string& context, const Json& options, const std::string& chosen,
                  const std::string& reasoning, const std::string& level, const std::string& model);
  bool update_outcome(const std::string& id, const std::string& outcome);
  double success_rate(const std::string& context_substr);
  Json recent(int n);
  size_t size();

 private:
  std::mutex mu_;
  std::deque<Json> ring_;
  size_t cap_;
};

class ResultAggregator {
 public:
  void record(const std::string& goal_id, const Json& result);
  Json summary(const std::string& goal_id);
  Json results(const std::string& goal_id);

 private:
  std::mutex mu_;
  std::map<std::string, std::vector<Json>> by_goal_;
};

bool cron_matches(const std::string& expr, int64_t unix_time);
bool cron_valid(const std::string& expr);

class ScheduleStore {
 public:
  explicit ScheduleStore(const std::string& db_path);
  std::string create(const std::string& cron, const std::string& goal_template, int priority);
  Json list();
  bool remove(const std::string& id);
  Json due(int64_t now);  // entries matching this minute, marked as run (at most once per minute)

 private:
  std::mutex mu_;
  Db db_;
};

class EventBus {
 public:
  std::string subscribe(const std::string& event_pattern, const std::string& min_severity,
                        const std::string& goal_template, int priority);
  bool unsubscribe(const std::string& id);
  // returns [{description, priority, subscription_id}] goals to create for this event
  Json publish(const Json& event);
  Json recent(int n);

 private:
  static int sev(const std::string& s);
  std::mutex mu_;
  std::vector<Json> subs_;
  std::deque<Json> events_;
};

std::string build_system_prompt(const std::string& task, const std::string& level, const Json& tools,
                                const Json& patterns, int max_tokens);

}  // namespace aiosn
