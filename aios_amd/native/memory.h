// Four-tier memory core (MI355X build of the reference's `memory/` crate):
//   operational (hot)  : ring buffer of 10,000 events + metrics map        (operational.rs)
//   working (warm)     : SQLite goals/tasks/tool_calls/decisions/patterns/agent_states (working.rs)
//   long-term (cold)   : SQLite procedures (64-d hashed embedding)/incidents/config_changes (longterm.rs)
//   knowledge          : hybrid keyword + embedding search (knowledge.rs; persisted here, the
//                        reference kept it in an in-memory DB and lost it on restart -- App. A)
// plus the tier-migration pipeline (migration.rs, started by the service here) and
// AssembleContext (main.rs:353-480, 4 chars/token budget, relevance-sorted chunks).
// Records cross the binding as JSON objects with the proto field names.
#pragma once
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "json.h"
#include "util.h"

namespace aiosn {

std::vector<float> hashed_embedding(const std::string& text, int dim = 64);
double cosine(const std::vector<float>& a, const std::vector<float>& b);
double keyword_relevance(const std::vector<std::string>& keywords, const std::string& text);
int estimate_tokens(const std::string& s);

class OperationalMemory {
 public:
  explicit OperationalMemory(size_t cap = 10000) : cap_(cap) {}
  void push_event(Json ev);
  Json recent(int count, const std::string& category, const std::string& source) const;
  void update_metric(const std::string& key, double value, int64_t ts);
  bool metric(const std::string& key, double& value, int64_t& ts) const;
  Json snapshot() const;
  size_t size() const;

 private:
  size_t cap_;
  mutable std::mutex mu_;
  std::deque<Json> events_;
  std::map<std::string, std::pair<double, int64_t>> metrics_;
};

class MemoryStore {
 public:
  MemoryStore(const std::string& working_db, const std::string& longterm_db, const std::string& knowledge_db);

  OperationalMemory& operational() { return op_; }

  // working
  void store_goal(const Json& g);
  void update_goal(const std::string& id, const std::string& status, const std::string& result);
  Json active_goals();
  void store_task(const Json& t);
  Json tasks_for_goal(const std::string& goal_id);
  void store_tool_call(const Json& c);
  void store_decision(const Json& d);
  void store_pattern(const Json& p);
  Json find_pattern(const std::string& trigger, double min_success);  // {} if none
  void update_pattern_stats(const std::string& id, bool success);
  void store_agent_state(const std::string& agent, const std::string& state_json);
  Json agent_state(const std::string& agent);
  Json learn_pattern_from_goal(const std::string& goal_id);
  Json tool_sequence_for_goal(const std::string& goal_id);

  // long-term
  void store_procedure(const Json& p);
  void store_incident(const Json& i);
  void store_config_change(const Json& c);
  Json semantic_search(const std::string& query, const std::vector<std::string>& collections, int n, double min_rel);

  // knowledge
  void add_knowledge(const Json& k);
  Json search_knowledge(const std::string& query, int n, double min_rel);

  // context assembly
  Json assemble_context(const std::string& task, int max_tokens, const std::vector<std::string>& tiers);

  // migration (migration.rs): completed goals older than max_goal_age_s -> procedures; patterns
  // capped at max_patterns (worst first); tool calls older than max_call_age_s deleted
  Json migrate(int64_t max_goal_age_s = 3600, int max_patterns = 1000, int64_t max_call_age_s = 48 * 3600);

  Json stats();

 private:
  OperationalMemory op_;
  Db work_, lt_, kn_;
};

}  // namespace aiosn
