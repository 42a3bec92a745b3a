// Tool registry + execution pipeline core (MI355X build of the reference's `tools/` crate).
//
// Behaviour follows the reference: registry of ToolDefinitions, least-privilege
// capability checks (`tools/src/capabilities.rs:51-378`), token-bucket rate limiting 10 rps per
// agent / 50 rps per tool with burst x2 (`executor.rs:19-84`), pre-execution backups for
// reversible fs tools (`backup.rs:36-94`), SHA-256 hash-chained audit ledger in SQLite
// (`audit.rs:15-107`), sandboxed plugin scripts with rlimits (`sandbox.rs:112-205`), plugin
// chaining pipe/merge (`main.rs:177-244`) and the 88 built-in tools in 16 namespaces.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "json.h"
#include "util.h"

namespace aiosn {

struct ToolDef {
  std::string name, ns, version = "1.0.0", description;
  std::vector<std::string> required_caps;  // registry metadata (dotted, as the reference registry)
  std::string risk_level;                  // low | medium | high | critical
  bool requires_confirmation = false;
  bool idempotent = false, reversible = false;
  int timeout_ms = 5000;
  std::string rollback_tool;
  std::string handler_address;             // externally registered tools (Register RPC)
  std::string input_schema;                // JSON schema of the input ("" = unchecked); see security.h
};

struct CapCheck {
  bool allowed = false;
  std::string reason, risk;
  std::vector<std::string> missing;
};

class CapabilityChecker {
 public:
  CapabilityChecker();
  CapCheck check(const std::string& agent, const std::string& tool) const;
  void register_agent(const std::string& agent, const std::vector<std::string>& caps);
  void grant(const std::string& agent, const std::vector<std::string>& caps);
  int revoke(const std::string& agent, const std::vector<std::string>& caps, bool all);
  void set_requirement(const std::string& tool, const std::vector<std::string>& caps, const std::string& risk);
  std::vector<std::string> agent_caps(const std::string& agent) const;
  static const std::vector<std::string>& all_capabilities();

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::set<std::string>> agents_;
  std::map<std::string, std::pair<std::vector<std::string>, std::string>> req_;
};

class RateLimiter {
 public:
  RateLimiter(double agent_rps = 10, double tool_rps = 50) : agent_rps_(agent_rps), tool_rps_(tool_rps) {}
  bool check(const std::string& agent, const std::string& tool);

 private:
  struct Bucket {
    double tokens, max, rate;
    int64_t last_ms;
  };
  bool take(std::map<std::string, Bucket>& m, const std::string& k, double rps);
  std::mutex mu_;
  std::map<std::string, Bucket> agents_, tools_;
  double agent_rps_, tool_rps_;
};

class AuditLog {
 public:
  explicit AuditLog(const std::string& db_path);
  void record(const std::string& execution_id, const std::string& tool, const std::string& agent,
              const std::string& task, const std::string& reason, bool success, int64_t duration_ms);
  bool verify_chain();
  Json query(const std::string& tool, const std::string& agent, const std::string& since, const std::string& until,
             int limit);
  int64_t count();

 private:
  Db db_;
  std::string last_hash_;
  std::mutex mu_;
};

class BackupManager {
 public:
  explicit BackupManager(const std::string& dir);
  std::string create_backup(const std::string& execution_id, const std::string& tool, const std::string& input_json);
  bool rollback(const std::string& execution_id);
  int cleanup_old(int64_t max_age_s);
  const std::string& dir() const { return dir_; }

 private:
  struct Entry {
    std::string tool, backup_path, input, target;
    bool existed = false;
    int64_t created = 0;
  };
  std::string dir_;
  std::mutex mu_;
  std::map<std::string, Entry> entries_;
};

struct SandboxLimits {
  size_t mem_bytes = 256ull << 20;
  int cpu_seconds = 30;
  int max_fds = 64;
  int max_procs = 16;
  bool allow_network = false;
  std::vector<std::string> writable_paths{"/tmp"};
  int timeout_ms = 30000;
};
struct SandboxResult {
  bool success = false;
  std::string output, error;
  int exit_code = -1;
  int64_t duration_ms = 0;
};
SandboxResult sandbox_exec(const std::string& cmd, const std::vector<std::string>& args, const std::string& input,
                           const SandboxLimits& lim);
// tools/src/sandbox.rs:208-215 -- tools that should run inside the sandbox
bool should_sandbox(const std::string& tool, const std::string& risk);

struct ExecResult {
  bool success = false;
  std::string output_json, error, execution_id, backup_id;
  int64_t duration_ms = 0;
};

struct ToolContext;  // handlers' view of the service (audit, checker, plugin dir, ...)
using ToolHandler = std::function<Json(const Json& input, ToolContext& ctx)>;

struct ToolPaths {
  std::string data_dir = "/var/lib/aios";
  std::string audit_db() const { return data_dir + "/ledger/audit.db"; }
  std::string backup_dir() const { return data_dir + "/cache/backups"; }
  std::string plugin_dir() const { return data_dir + "/plugins"; }
  std::string integrity_db() const { return data_dir + "/ledger/integrity.db"; }
  std::string grants_db() const { return data_dir + "/ledger/grants.db"; }
  std::string source_dir;  // self.* tools (AIOS_SOURCE_DIR)
};

class ToolService {
 public:
  explicit ToolService(const ToolPaths& paths);
  ~ToolService();

  std::vector<ToolDef> list_tools(const std::string& ns) const;
  bool get_tool(const std::string& name, ToolDef& out) const;
  bool register_tool(const ToolDef& def, std::string& err);
  bool deregister_tool(const std::string& name);
  ExecResult execute(const std::string& tool, const std::string& agent, const std::string& task,
                     const std::string& input_json, const std::string& reason);
  bool rollback(const std::string& execution_id, std::string& err);
  int scan_plugins();
  size_t tool_count() const;
  CapabilityChecker& caps() { return caps_; }
  AuditLog& audit() { return *audit_; }
  const ToolPaths& paths() const { return paths_; }
  void set_handler(const std::string& tool, ToolHandler h);

 private:
  ExecResult run_pipeline(const std::string& tool, const std::string& agent, const std::string& task,
                          const std::string& input_json, const std::string& reason, bool audit_it);
  void register_builtins();

  ToolPaths paths_;
  mutable std::mutex mu_;
  std::map<std::string, ToolDef> tools_;
  std::map<std::string, ToolHandler> handlers_;
  CapabilityChecker caps_;
  RateLimiter limiter_;
  std::unique_ptr<AuditLog> audit_;
  std::unique_ptr<BackupManager> backups_;
  std::unique_ptr<ToolContext> ctx_;
};

struct ToolContext {
  ToolService* svc;
  const ToolPaths* paths;
};

// handler registration per namespace group (tools_*.cpp)
struct ToolSpec {
  ToolDef def;
  std::vector<std::string> caps;  // capability-checker requirement (underscore names)
  ToolHandler fn;
};
void add_fs_process_service_tools(std::vector<ToolSpec>& out);
void add_system_tools(std::vector<ToolSpec>& out);
void add_dev_tools(std::vector<ToolSpec>& out);

// plugin helpers (tools_dev.cpp)
Json plugin_validate(const std::string& code);
std::string plugin_wrapper(const std::string& user_code);

// shared helpers for handlers
[[noreturn]] void tool_fail(const std::string& msg);
std::string req_str(const Json& in, const char* key);
std::string abs_path(const Json& in, const char* key);

}  // namespace aiosn
