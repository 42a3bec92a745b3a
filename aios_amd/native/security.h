// Security and plugin-runtime pieces of the tools crate that the reference defines but never
// wires (SURVEY.md §2.4 "Wired? no" rows) plus the orchestrator's mTLS manager (§2.2):
//   toml_parse          TOML subset incl. [[array of tables]]            (the crates' toml use)
//   SecretManager       secrets.toml cache with TTL, 0600 check, wipe     (tools/src/secrets.rs)
//   FirewallApplicator  firewall-rules.toml -> nft / iptables, dry run,
//                       apply, rollback                                   (tools/src/firewall_apply.rs)
//   schema_validate     JSON-schema subset for tool inputs                (tools/src/schema.rs)
//   TriggerStore        plugin triggers (cron, file_watch, log_pattern,
//                       metric_threshold) persisted in SQLite + checks    (tools/src/plugin/{events,triggers}.rs)
//   PluginWatcher       plugin-dir change detection for hot reload        (tools/src/plugin/mod.rs:167-219)
//   TlsManager          self-signed CA + server certificate (OpenSSL)     (agent-core/src/tls.rs)
// Here they are wired: tool inputs are schema-checked in the executor pipeline, the tools
// daemon runs the watcher/trigger loop, the gateway reads provider keys through SecretManager.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.h"

namespace aiosn {

class Db;  // util.h

Json toml_parse(const std::string& text);  // throws std::runtime_error on malformed headers

// ------------------------------------------------------------------------------ secrets
class SecretManager {
 public:
  explicit SecretManager(const std::string& path, int ttl_s = 3600) : path_(path), ttl_s_(ttl_s) {}
  ~SecretManager() { wipe(); }
  // (re)load the file: top-level string keys and one level of tables ("api_keys.claude");
  // returns the number of secrets cached; insecure permissions (not 0600) are reported in warnings()
  int load();
  bool get(const std::string& key, std::string& out) const;  // false if missing or expired
  std::string get_or_reload(const std::string& key);          // reload once on a miss / expiry
  void set(const std::string& key, const std::string& value);
  void wipe();  // zero every cached value, then drop them
  size_t count() const { return cache_.size(); }
  // provider keys: secrets file first, then the environment (CLAUDE_API_KEY, OPENAI_API_KEY, QWEN3_API_KEY)
  Json api_keys();
  const std::vector<std::string>& warnings() const { return warnings_; }

 private:
  struct Entry {
    std::string value;
    int64_t loaded_ms;
  };
  std::string path_;
  int ttl_s_;
  std::map<std::string, Entry> cache_;
  std::vector<std::string> warnings_;
};

// ------------------------------------------------------------------------------ firewall
struct FirewallRule {
  std::string name, action, direction, protocol, source, destination, interface, comment;
  int port = 0, port_lo = 0, port_hi = 0;
  std::vector<std::string> state;  // conntrack states (established, related, ...)
  std::string raw;                 // raw nft rule expression ({chain, rule} layout), nft only
};

class FirewallApplicator {
 public:
  // backend "nft", "iptables" or "auto" (nft when the binary exists)
  explicit FirewallApplicator(const std::string& config_path, const std::string& backend = "auto");
  // rules from either layout: [[rules]] with direction = "input" | ... or [[input]] / [[output]] /
  // [[forward]] tables; [defaults] *_policy (or default_policy) give chain policies
  std::vector<FirewallRule> load_config(std::map<std::string, std::string>* policies = nullptr) const;
  std::string to_nftables(const FirewallRule& r) const;
  std::string to_iptables(const FirewallRule& r) const;
  std::string command(const FirewallRule& r) const { return nft_ ? to_nftables(r) : to_iptables(r); }
  std::vector<std::string> setup_commands() const;     // table/chains (+ policies) for nft
  std::vector<std::string> dry_run() const;            // setup + one command per rule
  // run the commands (dry_run=false needs root + the backend); applied rules are recorded
  Json apply(bool dry_run);
  void record_applied(const FirewallRule& r);
  std::vector<std::string> rollback_commands() const;  // newest first: add->delete, -A->-D
  size_t applied_count() const { return applied_.size(); }
  bool uses_nftables() const { return nft_; }

 private:
  std::string path_;
  bool nft_;
  std::vector<std::string> applied_;
};

// ------------------------------------------------------------------------------ schema
// Validates `v` against a JSON-schema subset: type (incl. arrays of types, "integer"), required,
// properties, additionalProperties (bool or schema), enum, const, minimum / maximum /
// exclusiveMinimum / exclusiveMaximum, minLength / maxLength, pattern, items, minItems /
// maxItems, anyOf / oneOf / allOf.  Returns one message per violation ("$.path: reason").
std::vector<std::string> schema_validate(const Json& v, const Json& schema);

// ------------------------------------------------------------------------------ triggers
bool trigger_check_cron(const std::string& expr, int64_t unix_time);
bool trigger_check_file_watch(const std::string& path, int64_t last_checked);  // mtime > last_checked
bool trigger_check_metric(double value, const std::string& op, double threshold);
bool trigger_check_log_pattern(const std::string& line, const std::string& pattern);  // regex, substring fallback

struct PluginTrigger {
  std::string id, plugin, type;  // type: cron | file_watch | log_pattern | metric_threshold
  Json config;                   // {expression} | {path} | {pattern, log_path} | {metric, operator, threshold}
  bool enabled = true;
  int64_t last_fired = 0;
};

class TriggerStore {
 public:
  explicit TriggerStore(const std::string& db_path);  // ":memory:" allowed
  ~TriggerStore();
  std::string add(const std::string& plugin, const std::string& type, const Json& config);  // throws on bad config
  bool remove(const std::string& id);
  bool set_enabled(const std::string& id, bool enabled);
  std::vector<PluginTrigger> list() const;
  // evaluate every enabled trigger at `now` against the metric snapshot (name -> value) and the
  // new log lines per log path; returns the triggers that fire (last_fired is updated; a cron
  // trigger fires at most once per minute)
  std::vector<PluginTrigger> due(int64_t now, const Json& metrics, const Json& log_lines);

 private:
  void save(const PluginTrigger& t);
  std::unique_ptr<Db> db_;
  std::map<std::string, PluginTrigger> triggers_;
};

// ------------------------------------------------------------------------------ plugin watcher
class PluginWatcher {
 public:
  explicit PluginWatcher(const std::string& dir) : dir_(dir) {}
  // compare the *.py / *.meta.json mtimes with the previous poll: {"added", "changed", "removed"}
  Json poll();

 private:
  std::string dir_;
  std::map<std::string, int64_t> seen_;
  bool first_ = true;
};

// ------------------------------------------------------------------------------ TLS
class TlsManager {
 public:
  explicit TlsManager(const std::string& cert_dir) : dir_(cert_dir) {}
  bool certs_exist() const;
  // CA (EC P-256, 10 y) + server certificate for `service` (SAN: localhost, 127.0.0.1, service),
  // signed by the CA; idempotent: existing files are kept.  Returns the paths.
  Json generate_self_signed(const std::string& service, int days = 365);
  // files exist, parse, server cert is signed by the CA and inside its validity window
  Json verify() const;
  Json paths() const;

 private:
  std::string dir_;
};

}  // namespace aiosn
