// Tool service core: capability checker, rate limiter, audit ledger, backups, sandbox, pipeline.
// Reference behaviour: tools/src/{capabilities,executor,audit,backup,sandbox,main}.rs.
#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>

#include "tools.h"
#include "security.h"

namespace aiosn {

[[noreturn]] void tool_fail(const std::string& msg) { throw std::runtime_error(msg); }

std::string req_str(const Json& in, const char* key) {
  const Json& v = in[key];
  if (!v.is_str() || v.as_str().empty()) tool_fail(std::string("missing required field '") + key + "'");
  return v.as_str();
}

std::string abs_path(const Json& in, const char* key) {
  std::string p = req_str(in, key);
  if (p[0] != '/') tool_fail(std::string("'") + key + "' must be an absolute path: " + p);
  return p;
}

// ------------------------------------------------------------------------------ capabilities
const std::vector<std::string>& CapabilityChecker::all_capabilities() {
  // tools/src/capabilities.rs:53-84 (30 capability strings)
  static const std::vector<std::string> all = {
      "fs_read",       "fs_write",        "fs_delete",      "fs_permissions", "process_read",  "process_manage",
      "service_read",  "service_manage",  "net_read",       "net_write",      "net_scan",      "firewall_read",
      "firewall_manage", "pkg_read",      "pkg_manage",     "sec_read",       "sec_manage",    "monitor_read",
      "hw_read",       "git_read",        "git_write",      "code_gen",       "self_read",     "self_update",
      "plugin_read",   "plugin_manage",   "plugin_execute", "container_read", "container_manage", "email_send"};
  return all;
}

CapabilityChecker::CapabilityChecker() {
  // 11 built-in principals (capabilities.rs:51-191)
  register_agent("autonomy-loop", all_capabilities());
  register_agent("task-agent", all_capabilities());
  register_agent("system-agent", {"monitor_read", "service_read", "service_manage", "process_read"});
  register_agent("network-agent", {"net_read", "net_write", "net_scan", "firewall_read", "firewall_manage"});
  register_agent("security-agent",
                 {"sec_read", "sec_manage", "net_read", "net_scan", "process_read", "monitor_read", "fs_read"});
  register_agent("monitoring-agent", {"monitor_read", "net_read", "process_read", "fs_read", "hw_read"});
  register_agent("storage-agent",
                 {"fs_read", "fs_write", "fs_delete", "fs_permissions", "monitor_read", "process_manage"});
  register_agent("package-agent", {"pkg_read", "pkg_manage"});
  register_agent("learning-agent", {"monitor_read", "process_read", "fs_read"});
  register_agent("creator-agent", {"fs_read", "fs_write", "code_gen", "git_read", "git_write", "process_manage",
                                   "plugin_read", "plugin_manage", "plugin_execute"});
  register_agent("web-agent", {"net_read", "net_write", "fs_read", "fs_write"});
}

void CapabilityChecker::register_agent(const std::string& agent, const std::vector<std::string>& caps) {
  std::lock_guard<std::mutex> g(mu_);
  agents_[agent] = std::set<std::string>(caps.begin(), caps.end());
}
void CapabilityChecker::grant(const std::string& agent, const std::vector<std::string>& caps) {
  std::lock_guard<std::mutex> g(mu_);
  auto& s = agents_[agent];
  s.insert(caps.begin(), caps.end());
}
int CapabilityChecker::revoke(const std::string& agent, const std::vector<std::string>& caps, bool all) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = agents_.find(agent);
  if (it == agents_.end()) return 0;
  if (all) {
    const int n = (int)it->second.size();
    it->second.clear();
    return n;
  }
  int n = 0;
  for (auto& c : caps) n += (int)it->second.erase(c);
  return n;
}
void CapabilityChecker::set_requirement(const std::string& tool, const std::vector<std::string>& caps,
                                        const std::string& risk) {
  std::lock_guard<std::mutex> g(mu_);
  req_[tool] = {caps, risk};
}
std::vector<std::string> CapabilityChecker::agent_caps(const std::string& agent) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = agents_.find(agent);
  if (it == agents_.end()) return {};
  return std::vector<std::string>(it->second.begin(), it->second.end());
}

CapCheck CapabilityChecker::check(const std::string& agent, const std::string& tool) const {
  std::lock_guard<std::mutex> g(mu_);
  CapCheck r;
  auto rq = req_.find(tool);
  auto ag = agents_.find(agent);
  if (rq == req_.end()) {
    // dynamically created plugin tools need plugin_execute (capabilities.rs:394-417)
    if (starts_with(tool, "plugin.")) {
      r.risk = "medium";
      if (ag != agents_.end() && ag->second.count("plugin_execute")) {
        r.allowed = true;
        r.reason = "Dynamic plugin tool - agent has plugin_execute capability";
      } else {
        r.reason = "Dynamic plugin tool " + tool + " requires plugin_execute capability";
        r.missing = {"plugin_execute"};
      }
      return r;
    }
    r.risk = "critical";
    r.reason = "No capability requirement defined for tool: " + tool;  // deny by default
    return r;
  }
  r.risk = rq->second.second;
  if (ag == agents_.end()) {
    r.reason = "Agent " + agent + " has no registered capabilities";
    r.missing = rq->second.first;
    return r;
  }
  for (auto& c : rq->second.first)
    if (!ag->second.count(c)) r.missing.push_back(c);
  r.allowed = r.missing.empty();
  r.reason = r.allowed ? "All required capabilities present" : "Missing capabilities";
  return r;
}

// ------------------------------------------------------------------------------ rate limiting
bool RateLimiter::take(std::map<std::string, Bucket>& m, const std::string& k, double rps) {
  const int64_t now = now_ms();
  auto it = m.find(k);
  if (it == m.end()) it = m.emplace(k, Bucket{rps * 2.0, rps * 2.0, rps, now}).first;  // burst x2
  Bucket& b = it->second;
  b.tokens = std::min(b.max, b.tokens + (double)(now - b.last_ms) / 1000.0 * b.rate);
  b.last_ms = now;
  if (b.tokens >= 1.0) {
    b.tokens -= 1.0;
    return true;
  }
  return false;
}
bool RateLimiter::check(const std::string& agent, const std::string& tool) {
  std::lock_guard<std::mutex> g(mu_);
  const bool a = take(agents_, agent, agent_rps_);
  const bool t = take(tools_, tool, tool_rps_);
  return a && t;
}

// ------------------------------------------------------------------------------ audit ledger
AuditLog::AuditLog(const std::string& db_path) : db_(db_path) {
  db_.exec(
      "CREATE TABLE IF NOT EXISTS audit_log (id INTEGER PRIMARY KEY AUTOINCREMENT, execution_id TEXT NOT NULL,"
      " tool_name TEXT NOT NULL, agent_id TEXT NOT NULL, task_id TEXT NOT NULL, reason TEXT NOT NULL,"
      " success INTEGER NOT NULL, duration_ms INTEGER NOT NULL, timestamp TEXT NOT NULL, prev_hash TEXT NOT NULL,"
      " hash TEXT NOT NULL);"
      "CREATE INDEX IF NOT EXISTS idx_audit_tool ON audit_log(tool_name);"
      "CREATE INDEX IF NOT EXISTS idx_audit_agent ON audit_log(agent_id);"
      "CREATE INDEX IF NOT EXISTS idx_audit_time ON audit_log(timestamp);");
  Stmt s(db_, "SELECT hash FROM audit_log ORDER BY id DESC LIMIT 1");
  last_hash_ = s.step() ? s.col_text(0) : "genesis";
}

void AuditLog::record(const std::string& execution_id, const std::string& tool, const std::string& agent,
                      const std::string& task, const std::string& reason, bool success, int64_t duration_ms) {
  std::lock_guard<std::mutex> g(mu_);
  const std::string ts = now_rfc3339();
  // SHA256(prev_hash || execution_id || tool || agent || timestamp)  (audit.rs:62-68)
  const std::string hash = sha256_hex(last_hash_ + execution_id + tool + agent + ts);
  try {
    Stmt s(db_,
           "INSERT INTO audit_log (execution_id, tool_name, agent_id, task_id, reason, success, duration_ms, timestamp,"
           " prev_hash, hash) VALUES (?1,?2,?3,?4,?5,?6,?7,?8,?9,?10)");
    s.bind(1, execution_id).bind(2, tool).bind(3, agent).bind(4, task).bind(5, reason);
    s.bind(6, (int64_t)(success ? 1 : 0)).bind(7, duration_ms).bind(8, ts).bind(9, last_hash_).bind(10, hash);
    s.exec();
    last_hash_ = hash;
  } catch (const std::exception&) {
    // an audit write failure never fails the tool call (audit.rs:96-99)
  }
}

bool AuditLog::verify_chain() {
  std::lock_guard<std::mutex> g(mu_);
  Stmt s(db_, "SELECT execution_id, tool_name, agent_id, timestamp, prev_hash, hash FROM audit_log ORDER BY id ASC");
  std::string prev = "genesis";
  while (s.step()) {
    if (s.col_text(4) != prev) return false;
    const std::string h = sha256_hex(prev + s.col_text(0) + s.col_text(1) + s.col_text(2) + s.col_text(3));
    if (h != s.col_text(5)) return false;
    prev = h;
  }
  return true;
}

int64_t AuditLog::count() {
  std::lock_guard<std::mutex> g(mu_);
  Stmt s(db_, "SELECT COUNT(*) FROM audit_log");
  return s.step() ? s.col_int(0) : 0;
}

Json AuditLog::query(const std::string& tool, const std::string& agent, const std::string& since,
                     const std::string& until, int limit) {
  std::lock_guard<std::mutex> g(mu_);
  std::string sql =
      "SELECT id, execution_id, tool_name, agent_id, task_id, reason, success, duration_ms, timestamp, hash FROM "
      "audit_log WHERE 1=1";
  if (!tool.empty()) sql += " AND tool_name = ?1";
  if (!agent.empty()) sql += " AND agent_id = ?2";
  if (!since.empty()) sql += " AND timestamp >= ?3";
  if (!until.empty()) sql += " AND timestamp <= ?4";
  sql += " ORDER BY id DESC LIMIT ?5";
  Stmt s(db_, sql);
  if (!tool.empty()) s.bind(1, tool);
  if (!agent.empty()) s.bind(2, agent);
  if (!since.empty()) s.bind(3, since);
  if (!until.empty()) s.bind(4, until);
  s.bind(5, (int64_t)(limit > 0 ? limit : 100));
  Json out = Json::array();
  while (s.step()) {
    Json e = Json::object();
    e.set("id", s.col_int(0));
    e.set("execution_id", s.col_text(1));
    e.set("tool_name", s.col_text(2));
    e.set("agent_id", s.col_text(3));
    e.set("task_id", s.col_text(4));
    e.set("reason", s.col_text(5));
    e.set("success", s.col_int(6) != 0);
    e.set("duration_ms", s.col_int(7));
    e.set("timestamp", s.col_text(8));
    e.set("hash", s.col_text(9));
    out.push(e);
  }
  return out;
}

// ------------------------------------------------------------------------------ backups
BackupManager::BackupManager(const std::string& dir) : dir_(dir) { mkdirs(dir_); }

static bool copy_file(const std::string& src, const std::string& dst) {
  std::ifstream in(src, std::ios::binary);
  if (!in) return false;
  std::ofstream out(dst, std::ios::binary | std::ios::trunc);
  if (!out) return false;
  out << in.rdbuf();
  return (bool)out;
}

std::string BackupManager::create_backup(const std::string& execution_id, const std::string& tool,
                                         const std::string& input_json) {
  const std::string id = uuid4();
  Entry e;
  e.tool = tool;
  e.input = input_json;
  e.created = now_unix();
  if (starts_with(tool, "fs.")) {
    Json in;
    if (Json::try_parse(input_json, in)) {
      // the object a reversible fs tool modifies: path, or destination/link for move/copy/symlink
      std::string target = in.get_str("path");
      if (target.empty()) target = in.get_str("destination");
      if (target.empty()) target = in.get_str("link");
      e.target = target;
      struct stat st;
      if (!target.empty() && ::stat(target.c_str(), &st) == 0 && S_ISREG(st.st_mode)) {
        const std::string bp = dir_ + "/" + id;
        if (copy_file(target, bp)) {
          e.backup_path = bp;
          e.existed = true;
        }
      } else if (!target.empty() && ::lstat(target.c_str(), &st) != 0) {
        e.existed = false;  // created by the tool: rollback removes it
      }
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  entries_[execution_id] = e;
  return id;
}

bool BackupManager::rollback(const std::string& execution_id) {
  Entry e;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = entries_.find(execution_id);
    if (it == entries_.end()) return false;
    e = it->second;
    entries_.erase(it);
  }
  if (e.target.empty()) return false;
  if (e.existed && !e.backup_path.empty() && file_exists(e.backup_path)) {
    if (!copy_file(e.backup_path, e.target)) return false;
    ::unlink(e.backup_path.c_str());
    return true;
  }
  if (!e.existed && file_exists(e.target)) {
    struct stat st;
    if (::lstat(e.target.c_str(), &st) == 0 && (S_ISREG(st.st_mode) || S_ISLNK(st.st_mode)))
      return ::unlink(e.target.c_str()) == 0;
    if (S_ISDIR(st.st_mode)) return ::rmdir(e.target.c_str()) == 0;
  }
  return false;
}

int BackupManager::cleanup_old(int64_t max_age_s) {
  std::lock_guard<std::mutex> g(mu_);
  const int64_t now = now_unix();
  int n = 0;
  for (auto it = entries_.begin(); it != entries_.end();) {
    if (now - it->second.created > max_age_s) {
      if (!it->second.backup_path.empty()) ::unlink(it->second.backup_path.c_str());
      it = entries_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  return n;
}

// ------------------------------------------------------------------------------ sandbox
SandboxResult sandbox_exec(const std::string& cmd, const std::vector<std::string>& args, const std::string& input,
                           const SandboxLimits& lim) {
  SandboxResult r;
  const int64_t t0 = now_ms();
  CmdLimits cl;
  cl.timeout_ms = lim.timeout_ms > 0 ? lim.timeout_ms : lim.cpu_seconds * 1000;
  cl.mem_bytes = lim.mem_bytes;
  cl.cpu_seconds = lim.cpu_seconds;
  cl.max_fds = lim.max_fds;
  cl.max_procs = 0;  // RLIMIT_NPROC is per-user: enforcing it would also count the service's own threads
  cl.clear_env = true;  // env cleared, PATH=/usr/bin:/bin (sandbox.rs:135-141)
  cl.env.push_back("HOME=/tmp");
  cl.env.push_back(std::string("AIOS_SANDBOX_NETWORK=") + (lim.allow_network ? "1" : "0"));
  cl.stdin_data = input;
  cl.cwd = "/tmp";
  std::vector<std::string> argv{cmd};
  argv.insert(argv.end(), args.begin(), args.end());
  CmdResult c = run_cmd(argv, cl);
  r.duration_ms = now_ms() - t0;
  r.exit_code = c.exit_code;
  r.output = c.out;
  if (c.timed_out) {
    r.error = "sandbox: time limit exceeded";
    r.success = false;
  } else {
    r.success = c.exit_code == 0;
    if (!c.err.empty()) {
      if (r.success) r.output += "\n--- stderr ---\n" + c.err;
      else r.error = c.err;
    }
    if (!r.success && r.error.empty()) r.error = "exit code " + std::to_string(c.exit_code);
  }
  return r;
}

bool should_sandbox(const std::string& tool, const std::string&) {
  for (const char* p : {"process.spawn", "pkg.install", "pkg.remove", "firewall."})
    if (starts_with(tool, p)) return true;
  return false;
}

// ------------------------------------------------------------------------------ service
ToolService::ToolService(const ToolPaths& paths) : paths_(paths) {
  audit_ = std::make_unique<AuditLog>(paths_.audit_db());
  backups_ = std::make_unique<BackupManager>(paths_.backup_dir());
  ctx_ = std::make_unique<ToolContext>(ToolContext{this, &paths_});
  mkdirs(paths_.plugin_dir());
  register_builtins();
  scan_plugins();
}
ToolService::~ToolService() = default;

void ToolService::register_builtins() {
  std::vector<ToolSpec> specs;
  add_fs_process_service_tools(specs);
  add_system_tools(specs);
  add_dev_tools(specs);
  std::lock_guard<std::mutex> g(mu_);
  for (auto& s : specs) {
    s.def.requires_confirmation = s.def.risk_level == "critical";
    tools_[s.def.name] = s.def;
    handlers_[s.def.name] = s.fn;
    caps_.set_requirement(s.def.name, s.caps, s.def.risk_level);
  }
}

void ToolService::set_handler(const std::string& tool, ToolHandler h) {
  std::lock_guard<std::mutex> g(mu_);
  handlers_[tool] = std::move(h);
}

std::vector<ToolDef> ToolService::list_tools(const std::string& ns) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ToolDef> out;
  for (auto& kv : tools_)
    if (ns.empty() || kv.second.ns == ns) out.push_back(kv.second);
  return out;
}
bool ToolService::get_tool(const std::string& name, ToolDef& out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = tools_.find(name);
  if (it == tools_.end()) return false;
  out = it->second;
  return true;
}
size_t ToolService::tool_count() const {
  std::lock_guard<std::mutex> g(mu_);
  return tools_.size();
}
bool ToolService::register_tool(const ToolDef& def, std::string& err) {
  if (def.name.empty() || def.name.find('.') == std::string::npos) {
    err = "tool name must be <namespace>.<action>";
    return false;
  }
  std::lock_guard<std::mutex> g(mu_);
  ToolDef d = def;
  if (d.ns.empty()) d.ns = d.name.substr(0, d.name.find('.'));
  d.requires_confirmation = d.requires_confirmation || d.risk_level == "critical";
  tools_[d.name] = d;
  return true;
}
bool ToolService::deregister_tool(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  handlers_.erase(name);
  return tools_.erase(name) > 0;
}

int ToolService::scan_plugins() {
  // /var/lib/aios/plugins/<name>.py + <name>.meta.json -> tool "plugin.<name>" (plugin/mod.rs:107)
  DIR* d = ::opendir(paths_.plugin_dir().c_str());
  if (!d) return 0;
  int n = 0;
  while (dirent* e = ::readdir(d)) {
    std::string f = e->d_name;
    if (!ends_with(f, ".meta.json")) continue;
    const std::string name = f.substr(0, f.size() - 10);
    Json meta;
    try {
      meta = Json::parse(read_file(paths_.plugin_dir() + "/" + f));
    } catch (...) {
      continue;
    }
    ToolDef def;
    def.name = meta.get_str("tool_name", "plugin." + name);
    def.ns = "plugin";
    def.description = meta.get_str("description");
    def.risk_level = "medium";
    def.timeout_ms = (int)meta.get_int("timeout_ms", 30000);
    for (auto& c : meta["capabilities"].as_arr()) def.required_caps.push_back(c.as_str());
    if (meta["input_schema"].is_obj()) def.input_schema = meta["input_schema"].dump();
    std::lock_guard<std::mutex> g(mu_);
    if (!tools_.count(def.name)) ++n;
    tools_[def.name] = def;
  }
  ::closedir(d);
  return n;
}

ExecResult ToolService::run_pipeline(const std::string& tool, const std::string& agent, const std::string& task,
                                     const std::string& input_json, const std::string& reason, bool audit_it) {
  ExecResult r;
  r.execution_id = uuid4();
  const int64_t t0 = now_ms();
  ToolDef def;
  // 1. validate
  if (!get_tool(tool, def)) {
    r.error = "Unknown tool: " + tool;
    r.duration_ms = now_ms() - t0;
    return r;
  }
  // 1b. input schema (tools/src/schema.rs, unwired in the reference): a tool that declares a
  //     schema rejects malformed input before any capability or side effect
  if (!def.input_schema.empty()) {
    Json schema, in = Json::object();
    if (Json::try_parse(def.input_schema, schema) && (input_json.empty() || Json::try_parse(input_json, in))) {
      auto errs = schema_validate(in, schema);
      if (!errs.empty()) {
        std::string msg;
        for (size_t i = 0; i < errs.size() && i < 5; ++i) msg += (i ? "; " : "") + errs[i];
        r.error = "Input validation failed: " + msg;
        r.duration_ms = now_ms() - t0;
        return r;
      }
    }
  }
  // 2. capability check (denials are audited)
  CapCheck cc = caps_.check(agent, tool);
  if (!cc.allowed) {
    std::string miss;
    for (auto& m : cc.missing) miss += (miss.empty() ? "" : ", ") + ("\"" + m + "\"");
    r.error = "Capability denied: missing [" + miss + "]" + (cc.missing.empty() ? " (" + cc.reason + ")" : "");
    r.duration_ms = now_ms() - t0;
    if (audit_it) audit_->record(r.execution_id, tool, agent, task, reason, false, r.duration_ms);
    return r;
  }
  // 3. rate limit
  if (!limiter_.check(agent, tool)) {
    r.error = "Rate limit exceeded";
    r.duration_ms = now_ms() - t0;
    return r;
  }
  // 4. pre-execution backup for reversible tools
  if (def.reversible) r.backup_id = backups_->create_backup(r.execution_id, tool, input_json);
  // 5. run
  ToolHandler h;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = handlers_.find(tool);
    if (it != handlers_.end()) h = it->second;
  }
  if (h) {
    try {
      Json in = Json::object();
      if (!input_json.empty() && !Json::try_parse(input_json, in)) tool_fail("input_json is not valid JSON");
      if (!in.is_obj()) in = Json::object({{"value", in}});
      Json out = h(in, *ctx_);
      r.output_json = out.dump();
      r.success = true;
    } catch (const std::exception& e) {
      r.error = e.what();
    }
  } else if (starts_with(tool, "plugin.")) {
    // plugin script in the sandbox (main.rs:121-168)
    const std::string script = paths_.plugin_dir() + "/" + tool.substr(7) + ".py";
    if (file_exists(script)) {
      SandboxLimits lim;
      lim.allow_network = true;
      lim.cpu_seconds = 30;
      lim.timeout_ms = std::max(def.timeout_ms, 1000);
      lim.mem_bytes = 512ull << 20;
      SandboxResult sr = sandbox_exec("python3", {script}, input_json.empty() ? "{}" : input_json, lim);
      r.success = sr.success;
      r.error = sr.error;
      std::string out = trim(sr.output);
      // the plugin runner prints exactly one JSON document as its last line
      const auto nl = out.rfind('\n');
      const std::string last = nl == std::string::npos ? out : out.substr(nl + 1);
      Json j;
      r.output_json = Json::try_parse(last, j) ? j.dump() : Json::object({{"output", out}}).dump();
    } else {
      r.error = "No handler registered for tool: " + tool;
    }
  } else if (!def.handler_address.empty()) {
    r.error = "Externally registered tool " + tool + " is served at " + def.handler_address;
  } else {
    r.error = "No handler registered for tool: " + tool;
  }
  r.duration_ms = now_ms() - t0;
  // 6. audit
  if (audit_it) audit_->record(r.execution_id, tool, agent, task, reason, r.success, r.duration_ms);
  return r;
}

ExecResult ToolService::execute(const std::string& tool, const std::string& agent, const std::string& task,
                                const std::string& input_json, const std::string& reason) {
  ExecResult r = run_pipeline(tool, agent, task, input_json, reason, true);
  if (r.success && tool == "plugin.create") scan_plugins();
  // plugin chaining (main.rs:177-244): next_plugins get this output (pipe) or input+output (merge)
  if (r.success && starts_with(tool, "plugin.") && tool != "plugin.create" && tool != "plugin.list" &&
      tool != "plugin.delete" && tool != "plugin.install_deps" && tool != "plugin.from_template") {
    const std::string meta_path = paths_.plugin_dir() + "/" + tool.substr(7) + ".meta.json";
    Json meta;
    if (file_exists(meta_path) && Json::try_parse(read_file(meta_path), meta)) {
      const auto& next = meta["next_plugins"].as_arr();
      if (!next.empty()) {
        std::string carry = r.output_json;
        if (meta.get_str("output_mode", "pipe") == "merge") {
          Json a, b;
          Json::try_parse(input_json, a);
          Json::try_parse(r.output_json, b);
          if (!a.is_obj()) a = Json::object();
          for (auto& kv : b.as_obj()) a.set(kv.first, kv.second);
          carry = a.dump();
        }
        Json chain = Json::array();
        for (auto& n : next) {
          std::string nt = n.as_str();
          if (!starts_with(nt, "plugin.")) nt = "plugin." + nt;
          ExecResult cr = run_pipeline(nt, agent, task, carry, "chained from " + tool, true);
          chain.push(Json::object({{"tool", nt}, {"success", cr.success}, {"error", cr.error}}));
          if (!cr.success) break;
          carry = cr.output_json;
        }
        Json out;
        Json::try_parse(carry, out);
        Json wrapped = Json::object({{"output", out}, {"chain", chain}});
        r.output_json = wrapped.dump();
      }
    }
  }
  return r;
}

bool ToolService::rollback(const std::string& execution_id, std::string& err) {
  if (!backups_->rollback(execution_id)) {
    err = "No rollback available for execution " + execution_id;
    return false;
  }
  return true;
}

}  // namespace aiosn
