// Implementation of security.h (see there for the reference mapping).
#include "security.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/file.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <regex>
#include <sstream>
#include <stdexcept>

#include "orchestrator.h"
#include "util.h"

namespace aiosn {

static std::string upper_copy(std::string s) {
  for (auto& c : s) c = (char)toupper((unsigned char)c);
  return s;
}

// ============================================================================== TOML
namespace {

std::string strip_toml_comment(const std::string& line) {
  char q = 0;
  for (size_t i = 0; i < line.size(); ++i) {
    const char c = line[i];
    if (q) {
      if (c == '\\' && q == '"') { ++i; continue; }
      if (c == q) q = 0;
      continue;
    }
    if (c == '"' || c == '\'') q = c;
    else if (c == '#') return line.substr(0, i);
  }
  return line;
}

int bracket_balance(const std::string& s) {
  int n = 0;
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (q) {
      if (c == '\\' && q == '"') { ++i; continue; }
      if (c == q) q = 0;
      continue;
    }
    if (c == '"' || c == '\'') q = c;
    else if (c == '[' || c == '{') ++n;
    else if (c == ']' || c == '}') --n;
  }
  return n;
}

Json toml_scalar(const std::string& raw);

// split a flat list "a, b, [c, d]" at top-level commas
std::vector<std::string> split_top(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  int depth = 0;
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (q) {
      cur += c;
      if (c == '\\' && q == '"' && i + 1 < s.size()) { cur += s[++i]; continue; }
      if (c == q) q = 0;
      continue;
    }
    if (c == '"' || c == '\'') { q = c; cur += c; continue; }
    if (c == '[' || c == '{') ++depth;
    if (c == ']' || c == '}') --depth;
    if (c == ',' && depth == 0) {
      if (!trim(cur).empty()) out.push_back(trim(cur));
      cur.clear();
      continue;
    }
    cur += c;
  }
  if (!trim(cur).empty()) out.push_back(trim(cur));
  return out;
}

Json toml_scalar(const std::string& raw) {
  const std::string s = trim(raw);
  if (s.empty()) return Json();
  if (s[0] == '"' || s[0] == '\'') {
    const char q = s[0];
    std::string out;
    for (size_t i = 1; i < s.size() && s[i] != q; ++i) {
      if (q == '"' && s[i] == '\\' && i + 1 < s.size()) {
        const char e = s[++i];
        out += e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e;
      } else {
        out += s[i];
      }
    }
    return Json(out);
  }
  if (s[0] == '[') {
    Json a = Json::array();
    const size_t end = s.rfind(']');
    for (auto& item : split_top(s.substr(1, end == std::string::npos ? std::string::npos : end - 1)))
      a.push(toml_scalar(item));
    return a;
  }
  if (s[0] == '{') {  // inline table
    Json o = Json::object();
    const size_t end = s.rfind('}');
    for (auto& kv : split_top(s.substr(1, end == std::string::npos ? std::string::npos : end - 1))) {
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) continue;
      std::string k = trim(kv.substr(0, eq));
      if (!k.empty() && (k[0] == '"' || k[0] == '\'')) k = k.substr(1, k.size() - 2);
      o.set(k, toml_scalar(kv.substr(eq + 1)));
    }
    return o;
  }
  if (s == "true") return Json(true);
  if (s == "false") return Json(false);
  std::string num;
  for (char c : s)
    if (c != '_') num += c;
  char* end = nullptr;
  if (num.find_first_of(".eE") == std::string::npos) {
    const long long x = strtoll(num.c_str(), &end, 0);
    if (end && *end == 0) return Json((int64_t)x);
  }
  const double d = strtod(num.c_str(), &end);
  if (end && *end == 0) return Json(d);
  return Json(s);  // bare word (dates etc.) kept as text
}

std::vector<std::string> key_path(const std::string& name) {
  std::vector<std::string> out;
  for (auto& p : split(name, '.')) {
    std::string k = trim(p);
    if (!k.empty() && (k[0] == '"' || k[0] == '\'')) k = k.substr(1, k.size() - 2);
    out.push_back(k);
  }
  return out;
}

// path navigation on a tree that is rebuilt on the way back (Json values are shared by
// reference-counted handles; set() replaces the child)
void set_path(Json& node, const std::vector<std::string>& path, size_t i, const Json& value, bool append) {
  const std::string& k = path[i];
  if (i + 1 == path.size()) {
    if (append) {
      Json arr = node.has(k) && node[k].is_arr() ? node[k] : Json::array();
      arr.push(value);
      node.set(k, arr);
    } else {
      node.set(k, value);
    }
    return;
  }
  Json child = node.has(k) ? node[k] : Json::object();
  if (child.is_arr()) {  // [[a]] then [a.b]: the last element of the array of tables
    if (child.size() == 0) child.push(Json::object());
    Json last = child[child.size() - 1];
    set_path(last, path, i + 1, value, append);
    Json rebuilt = Json::array();
    for (size_t j = 0; j + 1 < child.size(); ++j) rebuilt.push(child[j]);
    rebuilt.push(last);
    node.set(k, rebuilt);
    return;
  }
  if (!child.is_obj()) child = Json::object();
  set_path(child, path, i + 1, value, append);
  node.set(k, child);
}

// [a.b] header: create missing tables along the path, keep existing ones
void ensure_table(Json& node, const std::vector<std::string>& path, size_t i) {
  if (i == path.size()) return;
  const std::string& k = path[i];
  Json child = node.has(k) ? node[k] : Json::object();
  if (child.is_arr()) {
    if (child.size() == 0) child.push(Json::object());
    Json last = child[child.size() - 1];
    ensure_table(last, path, i + 1);
    return;  // elements are shared handles: `last` already updated in place
  }
  if (!child.is_obj()) child = Json::object();
  ensure_table(child, path, i + 1);
  node.set(k, child);
}

}  // namespace

Json toml_parse(const std::string& text) {
  Json root = Json::object();
  std::vector<std::string> table;  // current table path ([[x]] -> the last element of x)
  std::istringstream in(text);
  std::string line, pending;
  int lineno = 0;
  while (std::getline(in, line)) {
    ++lineno;
    line = trim(strip_toml_comment(line));
    if (line.empty()) continue;
    if (!pending.empty()) {
      pending += " " + line;
      if (bracket_balance(pending) > 0) continue;
      line = pending;
      pending.clear();
    } else if (line[0] != '[' && line.find('=') != std::string::npos && bracket_balance(line) > 0) {
      pending = line;
      continue;
    }
    if (line[0] == '[') {
      const bool aot = line.size() > 1 && line[1] == '[';
      const size_t close = line.find(aot ? "]]" : "]");
      if (close == std::string::npos) throw std::runtime_error("toml: bad table header at line " + std::to_string(lineno));
      table = key_path(line.substr(aot ? 2 : 1, close - (aot ? 2 : 1)));
      if (aot) set_path(root, table, 0, Json::object(), true);
      else ensure_table(root, table, 0);
      continue;
    }
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::vector<std::string> kp = table;
    for (auto& k : key_path(line.substr(0, eq))) kp.push_back(k);
    if (kp.empty()) continue;
    // a [table] header created an empty object; keys under it merge into it
    set_path(root, kp, 0, toml_scalar(line.substr(eq + 1)), false);
  }
  return root;
}

// ============================================================================== secrets
int SecretManager::load() {
  warnings_.clear();
  struct stat st;
  if (::stat(path_.c_str(), &st) != 0) {
    warnings_.push_back("secrets file not found: " + path_);
    return 0;
  }
  if ((st.st_mode & 0777) != 0600) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%o", st.st_mode & 0777);
    warnings_.push_back(std::string("secrets file has insecure permissions ") + buf + " (expected 600)");
  }
  const Json t = toml_parse(read_file(path_));
  const int64_t now = now_ms();
  int n = 0;
  for (auto& kv : t.as_obj()) {
    if (kv.second.is_str()) {
      cache_[kv.first] = Entry{kv.second.as_str(), now};
      ++n;
    } else if (kv.second.is_obj()) {
      for (auto& in : kv.second.as_obj())
        if (in.second.is_str()) {
          cache_[kv.first + "." + in.first] = Entry{in.second.as_str(), now};
          ++n;
        }
    }
  }
  return n;
}

bool SecretManager::get(const std::string& key, std::string& out) const {
  auto it = cache_.find(key);
  if (it == cache_.end()) return false;
  if (now_ms() - it->second.loaded_ms >= (int64_t)ttl_s_ * 1000) return false;
  out = it->second.value;
  return true;
}

std::string SecretManager::get_or_reload(const std::string& key) {
  std::string v;
  if (get(key, v)) return v;
  load();
  return get(key, v) ? v : std::string();
}

void SecretManager::set(const std::string& key, const std::string& value) { cache_[key] = Entry{value, now_ms()}; }

void SecretManager::wipe() {
  for (auto& kv : cache_) {
    volatile char* p = &kv.second.value[0];
    for (size_t i = 0; i < kv.second.value.size(); ++i) p[i] = 0;
  }
  cache_.clear();
}

Json SecretManager::api_keys() {
  auto pick = [&](std::initializer_list<const char*> keys, const char* env) {
    for (const char* k : keys) {
      std::string v;
      if (get(k, v) && !v.empty()) return v;
    }
    return env_or(env, "");
  };
  return Json::object({{"claude", pick({"api_keys.claude", "claude_api_key", "anthropic_api_key"}, "CLAUDE_API_KEY")},
                       {"openai", pick({"api_keys.openai", "openai_api_key"}, "OPENAI_API_KEY")},
                       {"qwen3", pick({"api_keys.qwen3", "qwen3_api_key"}, "QWEN3_API_KEY")}});
}

// ============================================================================== firewall
FirewallApplicator::FirewallApplicator(const std::string& config_path, const std::string& backend)
    : path_(config_path) {
  if (backend == "nft") nft_ = true;
  else if (backend == "iptables") nft_ = false;
  else nft_ = have_cmd("nft") || !have_cmd("iptables");
}

static FirewallRule rule_from(const Json& j, const std::string& direction) {
  FirewallRule r;
  r.name = j.get_str("name");
  r.raw = j.get_str("rule");
  r.action = lower(j.get_str("action", "accept"));
  r.direction = lower(j.get_str("direction", j.get_str("chain", direction.empty() ? "input" : direction)));
  r.protocol = lower(j.get_str("protocol"));
  if (r.protocol == "all" || r.protocol == "any") r.protocol.clear();
  r.source = j.get_str("source");
  r.destination = j.get_str("destination");
  r.interface = j.get_str("interface");
  r.comment = j.get_str("comment", j.get_str("description"));
  r.port = (int)j.get_int("port", 0);
  const Json& pr = j["port_range"];
  if (pr.is_arr() && pr.size() == 2) {
    r.port_lo = (int)pr[0].as_int();
    r.port_hi = (int)pr[1].as_int();
  } else if (pr.is_str()) {
    auto p = split(pr.as_str(), '-');
    if (p.size() == 2) { r.port_lo = atoi(p[0].c_str()); r.port_hi = atoi(p[1].c_str()); }
  }
  const Json& st = j["state"];
  if (st.is_arr())
    for (auto& s : st.as_arr()) r.state.push_back(lower(s.as_str()));
  static const std::vector<std::string> actions = {"accept", "drop", "reject", "log"};
  static const std::vector<std::string> dirs = {"input", "output", "forward"};
  if (std::find(actions.begin(), actions.end(), r.action) == actions.end())
    throw std::runtime_error("firewall rule '" + r.name + "': bad action " + r.action);
  if (std::find(dirs.begin(), dirs.end(), r.direction) == dirs.end())
    throw std::runtime_error("firewall rule '" + r.name + "': bad direction " + r.direction);
  return r;
}

std::vector<FirewallRule> FirewallApplicator::load_config(std::map<std::string, std::string>* policies) const {
  std::vector<FirewallRule> out;
  if (!file_exists(path_)) return out;
  const Json t = toml_parse(read_file(path_));
  if (policies) {
    const Json& d = t["defaults"];
    // a single default_policy covers input and forward; output stays accept unless given
    // explicitly (a node that drops its own egress cannot reach its peers)
    for (const char* c : {"input", "output", "forward"}) {
      const std::string def = std::string(c) == "output" ? "" : t.get_str("default_policy");
      std::string p = d.get_str(std::string(c) + "_policy", def);
      if (!p.empty()) (*policies)[c] = lower(p);
    }
  }
  for (auto& r : t["rules"].as_arr()) out.push_back(rule_from(r, ""));
  for (const char* c : {"input", "output", "forward"})
    for (auto& r : t[c].as_arr()) out.push_back(rule_from(r, c));
  return out;
}

static std::string port_spec(const FirewallRule& r, const char* range_sep) {
  if (r.port) return std::to_string(r.port);
  if (r.port_lo && r.port_hi) return std::to_string(r.port_lo) + range_sep + std::to_string(r.port_hi);
  return "";
}

std::string FirewallApplicator::to_nftables(const FirewallRule& r) const {
  std::string cmd = "nft add rule inet aios " + r.direction;
  if (!r.raw.empty()) return cmd + " " + r.raw;
  if (!r.interface.empty()) {
    const bool neg = r.interface[0] == '!';
    const std::string ifn = neg ? r.interface.substr(1) : r.interface;
    cmd += std::string(r.direction == "output" ? " oifname " : " iifname ") + (neg ? "!= " : "") + "\"" + ifn + "\"";
  }
  if (!r.state.empty()) {
    cmd += " ct state ";
    for (size_t i = 0; i < r.state.size(); ++i) cmd += (i ? "," : "") + r.state[i];
  }
  if (!r.source.empty()) cmd += " ip saddr " + r.source;
  if (!r.destination.empty()) cmd += " ip daddr " + r.destination;
  if (!r.protocol.empty()) {
    const std::string ps = port_spec(r, "-");
    if (!ps.empty() && (r.protocol == "tcp" || r.protocol == "udp")) cmd += " " + r.protocol + " dport " + ps;
    else cmd += " meta l4proto " + r.protocol;
  }
  if (!r.comment.empty()) cmd += " comment \"" + r.comment + "\"";
  cmd += " " + r.action;
  return cmd;
}

std::string FirewallApplicator::to_iptables(const FirewallRule& r) const {
  std::string chain = upper_copy(r.direction);
  if (!r.raw.empty()) return "# nft-only rule (" + r.direction + "): " + r.raw;
  std::string cmd = "iptables -A " + chain;
  if (!r.interface.empty()) {
    const bool neg = r.interface[0] == '!';
    const std::string ifn = neg ? r.interface.substr(1) : r.interface;
    cmd += std::string(neg ? " !" : "") + (r.direction == "output" ? " -o " : " -i ") + ifn;
  }
  if (!r.protocol.empty()) {
    cmd += " -p " + r.protocol;
    const std::string ps = port_spec(r, ":");
    if (!ps.empty()) cmd += " --dport " + ps;
  }
  if (!r.state.empty()) {
    cmd += " -m conntrack --ctstate ";
    for (size_t i = 0; i < r.state.size(); ++i) cmd += (i ? "," : "") + upper_copy(r.state[i]);
  }
  if (!r.source.empty()) cmd += " -s " + r.source;
  if (!r.destination.empty()) cmd += " -d " + r.destination;
  cmd += " -j " + upper_copy(r.action);
  if (!r.comment.empty()) cmd += " -m comment --comment \"" + r.comment + "\"";
  return cmd;
}

std::vector<std::string> FirewallApplicator::setup_commands() const {
  std::map<std::string, std::string> pol;
  load_config(&pol);
  std::vector<std::string> out;
  if (nft_) {
    out.push_back("nft add table inet aios");
    for (const char* c : {"input", "output", "forward"}) {
      const std::string p = pol.count(c) ? pol[c] : "accept";
      out.push_back(std::string("nft add chain inet aios ") + c + " { type filter hook " + c +
                    " priority 0 ; policy " + p + " ; }");
    }
  } else {
    for (auto& kv : pol) out.push_back("iptables -P " + upper_copy(kv.first) + " " + upper_copy(kv.second));
  }
  return out;
}

std::vector<std::string> FirewallApplicator::dry_run() const {
  std::vector<std::string> out = setup_commands();
  for (auto& r : load_config()) out.push_back(command(r));
  return out;
}

Json FirewallApplicator::apply(bool dry) {
  Json res = Json::object();
  Json cmds = Json::array(), errors = Json::array();
  const auto rules = load_config();
  for (auto& c : setup_commands()) cmds.push(c);
  int applied = 0;
  if (!dry) {
    for (auto& c : setup_commands()) {
      CmdResult r = run_cmd({"/bin/sh", "-c", c});
      if (r.exit_code != 0) errors.push(c + ": " + trim(r.err));
    }
  }
  for (auto& rule : rules) {
    const std::string c = command(rule);
    cmds.push(c);
    if (dry || c[0] == '#') continue;
    CmdResult r = run_cmd({"/bin/sh", "-c", c});
    if (r.exit_code == 0) {
      record_applied(rule);
      ++applied;
    } else {
      errors.push(c + ": " + trim(r.err));
    }
  }
  res.set("dry_run", dry);
  res.set("backend", nft_ ? "nftables" : "iptables");
  res.set("commands", cmds);
  res.set("rules", (int64_t)rules.size());
  res.set("applied", (int64_t)applied);
  res.set("errors", errors);
  return res;
}

void FirewallApplicator::record_applied(const FirewallRule& r) { applied_.push_back(command(r)); }

std::vector<std::string> FirewallApplicator::rollback_commands() const {
  std::vector<std::string> out;
  for (auto it = applied_.rbegin(); it != applied_.rend(); ++it) {
    std::string c = *it;
    if (nft_) {
      const size_t p = c.find("add rule");
      if (p != std::string::npos) c.replace(p, 8, "delete rule");
    } else {
      const size_t p = c.find("-A ");
      if (p != std::string::npos) c.replace(p, 3, "-D ");
    }
    out.push_back(c);
  }
  return out;
}

// ============================================================================== schema
namespace {

std::string json_type(const Json& v) {
  if (v.is_null()) return "null";
  if (v.is_bool()) return "boolean";
  if (v.is_num()) return "number";
  if (v.is_str()) return "string";
  if (v.is_arr()) return "array";
  return "object";
}

bool type_ok(const Json& v, const std::string& t) {
  if (t == "integer") return v.is_num() && std::floor(v.as_num()) == v.as_num();
  if (t == "number") return v.is_num();
  return json_type(v) == t;
}

size_t utf8_len(const std::string& s) {
  size_t n = 0;
  for (unsigned char c : s)
    if ((c & 0xC0) != 0x80) ++n;
  return n;
}

void validate_at(const Json& v, const Json& s, const std::string& path, std::vector<std::string>& err) {
  if (!s.is_obj()) return;  // true / {} accept everything
  if (s.has("type")) {
    const Json& t = s["type"];
    bool ok = false;
    if (t.is_str()) ok = type_ok(v, t.as_str());
    else
      for (auto& x : t.as_arr()) ok = ok || type_ok(v, x.as_str());
    if (!ok) {
      err.push_back(path + ": expected type " + (t.is_str() ? t.as_str() : t.dump()) + ", got " + json_type(v));
      return;
    }
  }
  if (s.has("enum")) {
    bool ok = false;
    for (auto& e : s["enum"].as_arr()) ok = ok || e == v;
    if (!ok) err.push_back(path + ": value not in enum " + s["enum"].dump());
  }
  if (s.has("const") && !(s["const"] == v)) err.push_back(path + ": value must equal " + s["const"].dump());
  if (v.is_num()) {
    const double x = v.as_num();
    if (s.has("minimum") && x < s.get_num("minimum")) err.push_back(path + ": below minimum " + s["minimum"].dump());
    if (s.has("maximum") && x > s.get_num("maximum")) err.push_back(path + ": above maximum " + s["maximum"].dump());
    if (s.has("exclusiveMinimum") && x <= s.get_num("exclusiveMinimum"))
      err.push_back(path + ": not above exclusiveMinimum " + s["exclusiveMinimum"].dump());
    if (s.has("exclusiveMaximum") && x >= s.get_num("exclusiveMaximum"))
      err.push_back(path + ": not below exclusiveMaximum " + s["exclusiveMaximum"].dump());
  }
  if (v.is_str()) {
    const size_t n = utf8_len(v.as_str());
    if (s.has("minLength") && (int64_t)n < s.get_int("minLength")) err.push_back(path + ": shorter than minLength");
    if (s.has("maxLength") && (int64_t)n > s.get_int("maxLength")) err.push_back(path + ": longer than maxLength");
    if (s.has("pattern")) {
      try {
        if (!std::regex_search(v.as_str(), std::regex(s.get_str("pattern"))))
          err.push_back(path + ": does not match pattern " + s.get_str("pattern"));
      } catch (const std::regex_error&) {
        err.push_back(path + ": invalid pattern in schema");
      }
    }
  }
  if (v.is_arr()) {
    if (s.has("minItems") && (int64_t)v.size() < s.get_int("minItems")) err.push_back(path + ": fewer than minItems");
    if (s.has("maxItems") && (int64_t)v.size() > s.get_int("maxItems")) err.push_back(path + ": more than maxItems");
    if (s.has("items"))
      for (size_t i = 0; i < v.size(); ++i) validate_at(v[i], s["items"], path + "[" + std::to_string(i) + "]", err);
  }
  if (v.is_obj()) {
    for (auto& r : s["required"].as_arr())
      if (!v.has(r.as_str())) err.push_back(path + ": missing required property '" + r.as_str() + "'");
    const Json& props = s["properties"];
    for (auto& kv : v.as_obj()) {
      const std::string p = path + "." + kv.first;
      if (props.has(kv.first)) {
        validate_at(kv.second, props[kv.first], p, err);
      } else if (s.has("additionalProperties")) {
        const Json& ap = s["additionalProperties"];
        if (ap.is_bool() && !ap.as_bool()) err.push_back(path + ": unexpected property '" + kv.first + "'");
        else if (ap.is_obj()) validate_at(kv.second, ap, p, err);
      }
    }
  }
  if (s.has("allOf"))
    for (auto& sub : s["allOf"].as_arr()) validate_at(v, sub, path, err);
  if (s.has("anyOf") || s.has("oneOf")) {
    const bool one = s.has("oneOf");
    int matched = 0;
    for (auto& sub : s[one ? "oneOf" : "anyOf"].as_arr()) {
      std::vector<std::string> e2;
      validate_at(v, sub, path, e2);
      if (e2.empty()) ++matched;
    }
    if (one ? matched != 1 : matched == 0)
      err.push_back(path + (one ? ": must match exactly one schema in oneOf" : ": must match a schema in anyOf"));
  }
}

}  // namespace

std::vector<std::string> schema_validate(const Json& v, const Json& schema) {
  std::vector<std::string> err;
  validate_at(v, schema, "$", err);
  return err;
}

// ============================================================================== triggers
bool trigger_check_cron(const std::string& expr, int64_t t) { return cron_valid(expr) && cron_matches(expr, t); }

bool trigger_check_file_watch(const std::string& path, int64_t last_checked) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return false;
  return (int64_t)st.st_mtime > last_checked;
}

bool trigger_check_metric(double v, const std::string& op, double th) {
  if (op == ">" || op == "gt") return v > th;
  if (op == ">=" || op == "gte") return v >= th;
  if (op == "<" || op == "lt") return v < th;
  if (op == "<=" || op == "lte") return v <= th;
  if (op == "==" || op == "eq") return std::fabs(v - th) < 1e-9;
  if (op == "!=" || op == "ne") return std::fabs(v - th) >= 1e-9;
  return false;
}

bool trigger_check_log_pattern(const std::string& line, const std::string& pattern) {
  try {
    return std::regex_search(line, std::regex(pattern));
  } catch (const std::regex_error&) {
    return line.find(pattern) != std::string::npos;
  }
}

static void check_trigger_config(const std::string& type, const Json& c) {
  if (type == "cron") {
    if (!cron_valid(c.get_str("expression"))) throw std::runtime_error("cron trigger needs a valid 5-field 'expression'");
  } else if (type == "file_watch") {
    if (c.get_str("path").empty()) throw std::runtime_error("file_watch trigger needs 'path'");
  } else if (type == "log_pattern") {
    if (c.get_str("pattern").empty() || c.get_str("log_path").empty())
      throw std::runtime_error("log_pattern trigger needs 'pattern' and 'log_path'");
  } else if (type == "metric_threshold") {
    if (c.get_str("metric").empty() || c.get_str("operator").empty() || !c["threshold"].is_num())
      throw std::runtime_error("metric_threshold trigger needs 'metric', 'operator', numeric 'threshold'");
  } else {
    throw std::runtime_error("unknown trigger type: " + type);
  }
}

TriggerStore::TriggerStore(const std::string& db_path) : db_(new Db(db_path)) {
  db_->exec(
      "CREATE TABLE IF NOT EXISTS plugin_triggers (id TEXT PRIMARY KEY, plugin_name TEXT NOT NULL, "
      "trigger_type TEXT NOT NULL, config TEXT NOT NULL, enabled INTEGER NOT NULL DEFAULT 1, "
      "last_fired INTEGER NOT NULL DEFAULT 0)");
  Stmt st(*db_, "SELECT id, plugin_name, trigger_type, config, enabled, last_fired FROM plugin_triggers");
  while (st.step()) {
    PluginTrigger t;
    t.id = st.col_text(0);
    t.plugin = st.col_text(1);
    t.type = st.col_text(2);
    Json::try_parse(st.col_text(3), t.config);
    t.enabled = st.col_int(4) != 0;
    t.last_fired = st.col_int(5);
    triggers_[t.id] = t;
  }
}

TriggerStore::~TriggerStore() = default;

void TriggerStore::save(const PluginTrigger& t) {
  Stmt st(*db_,
          "INSERT OR REPLACE INTO plugin_triggers (id, plugin_name, trigger_type, config, enabled, last_fired) "
          "VALUES (?1, ?2, ?3, ?4, ?5, ?6)");
  st.bind(1, t.id).bind(2, t.plugin).bind(3, t.type).bind(4, t.config.dump());
  st.bind(5, (int64_t)(t.enabled ? 1 : 0)).bind(6, t.last_fired);
  st.exec();
}

std::string TriggerStore::add(const std::string& plugin, const std::string& type, const Json& config) {
  check_trigger_config(type, config);
  PluginTrigger t;
  t.id = uuid4();
  t.plugin = plugin;
  t.type = type;
  t.config = config;
  triggers_[t.id] = t;
  save(t);
  return t.id;
}

bool TriggerStore::remove(const std::string& id) {
  if (!triggers_.erase(id)) return false;
  Stmt st(*db_, "DELETE FROM plugin_triggers WHERE id = ?1");
  st.bind(1, id).exec();
  return true;
}

bool TriggerStore::set_enabled(const std::string& id, bool enabled) {
  auto it = triggers_.find(id);
  if (it == triggers_.end()) return false;
  it->second.enabled = enabled;
  save(it->second);
  return true;
}

std::vector<PluginTrigger> TriggerStore::list() const {
  std::vector<PluginTrigger> out;
  for (auto& kv : triggers_) out.push_back(kv.second);
  return out;
}

std::vector<PluginTrigger> TriggerStore::due(int64_t now, const Json& metrics, const Json& log_lines) {
  std::vector<PluginTrigger> out;
  for (auto& kv : triggers_) {
    PluginTrigger& t = kv.second;
    if (!t.enabled) continue;
    bool fire = false;
    if (t.type == "cron") {
      fire = now / 60 != t.last_fired / 60 && trigger_check_cron(t.config.get_str("expression"), now);
    } else if (t.type == "file_watch") {
      // first evaluation only records the baseline
      fire = t.last_fired > 0 && trigger_check_file_watch(t.config.get_str("path"), t.last_fired);
      if (t.last_fired == 0) {
        t.last_fired = now;
        save(t);
      }
    } else if (t.type == "log_pattern") {
      for (auto& line : log_lines[t.config.get_str("log_path")].as_arr())
        if (trigger_check_log_pattern(line.as_str(), t.config.get_str("pattern"))) { fire = true; break; }
    } else if (t.type == "metric_threshold") {
      const std::string m = t.config.get_str("metric");
      if (metrics.has(m))
        fire = trigger_check_metric(metrics[m].as_num(), t.config.get_str("operator"), t.config.get_num("threshold"));
    }
    if (fire) {
      t.last_fired = now;
      save(t);
      out.push_back(t);
    }
  }
  return out;
}

// ============================================================================== plugin watcher
Json PluginWatcher::poll() {
  std::map<std::string, int64_t> now;
  if (DIR* d = ::opendir(dir_.c_str())) {
    while (dirent* e = ::readdir(d)) {
      const std::string n = e->d_name;
      if (!ends_with(n, ".py") && !ends_with(n, ".meta.json")) continue;
      struct stat st;
      if (::stat((dir_ + "/" + n).c_str(), &st) == 0)
        now[n] = (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
    }
    ::closedir(d);
  }
  Json added = Json::array(), changed = Json::array(), removed = Json::array();
  auto plugin_of = [](const std::string& f) {
    return ends_with(f, ".meta.json") ? f.substr(0, f.size() - 10) : f.substr(0, f.size() - 3);
  };
  std::map<std::string, int> a, c, r;
  if (!first_) {
    for (auto& kv : now) {
      auto it = seen_.find(kv.first);
      if (it == seen_.end()) a[plugin_of(kv.first)] = 1;
      else if (it->second != kv.second) c[plugin_of(kv.first)] = 1;
    }
    for (auto& kv : seen_)
      if (!now.count(kv.first)) r[plugin_of(kv.first)] = 1;
  }
  for (auto& kv : a) added.push(kv.first);
  for (auto& kv : c)
    if (!a.count(kv.first)) changed.push(kv.first);
  for (auto& kv : r)
    if (!a.count(kv.first) && !c.count(kv.first)) removed.push(kv.first);
  seen_ = now;
  first_ = false;
  return Json::object({{"added", added}, {"changed", changed}, {"removed", removed},
                       {"total_files", (int64_t)now.size()}});
}

// ============================================================================== TLS
namespace {

struct PkeyDel { void operator()(EVP_PKEY* p) const { EVP_PKEY_free(p); } };
struct X509Del { void operator()(X509* p) const { X509_free(p); } };
using PkeyPtr = std::unique_ptr<EVP_PKEY, PkeyDel>;
using X509Ptr = std::unique_ptr<X509, X509Del>;

PkeyPtr ec_key() {
  EVP_PKEY* k = EVP_EC_gen("P-256");
  if (!k) throw std::runtime_error("tls: EC key generation failed");
  return PkeyPtr(k);
}

void add_ext(X509* cert, X509* issuer, int nid, const std::string& value) {
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, issuer, cert, nullptr, nullptr, 0);
  X509_EXTENSION* ex = X509V3_EXT_conf_nid(nullptr, &ctx, nid, value.c_str());
  if (!ex) throw std::runtime_error("tls: bad extension " + value);
  X509_add_ext(cert, ex, -1);
  X509_EXTENSION_free(ex);
}

X509Ptr make_cert(EVP_PKEY* key, const std::string& cn, X509* issuer, EVP_PKEY* issuer_key, int days, bool ca,
                  const std::string& san) {
  X509Ptr c(X509_new());
  X509_set_version(c.get(), 2);
  ASN1_INTEGER_set(X509_get_serialNumber(c.get()), (long)(now_ms() & 0x7fffffff));
  X509_gmtime_adj(X509_getm_notBefore(c.get()), -60);
  X509_gmtime_adj(X509_getm_notAfter(c.get()), (long)days * 86400L);
  X509_set_pubkey(c.get(), key);
  X509_NAME* name = X509_get_subject_name(c.get());
  X509_NAME_add_entry_by_txt(name, "O", MBSTRING_ASC, (const unsigned char*)"aiOS", -1, -1, 0);
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, (const unsigned char*)cn.c_str(), -1, -1, 0);
  X509_set_issuer_name(c.get(), issuer ? X509_get_subject_name(issuer) : name);
  X509* iss = issuer ? issuer : c.get();
  add_ext(c.get(), iss, NID_basic_constraints, ca ? "critical,CA:TRUE" : "critical,CA:FALSE");
  add_ext(c.get(), iss, NID_key_usage, ca ? "critical,keyCertSign,cRLSign" : "critical,digitalSignature,keyEncipherment");
  if (!san.empty()) add_ext(c.get(), iss, NID_subject_alt_name, san);
  if (!X509_sign(c.get(), issuer_key ? issuer_key : key, EVP_sha256())) throw std::runtime_error("tls: signing failed");
  return c;
}

// PEM files are written to a private temp file (created O_EXCL with the final mode, so a key is
// never world-readable, not even briefly) and rename()d into place: a concurrent reader sees the
// old file or the complete new one, never a half-written one.
FILE* open_private_tmp(const std::string& path, mode_t mode, std::string& tmp) {
  tmp = path + ".tmp." + std::to_string(::getpid());
  ::unlink(tmp.c_str());
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, mode);
  if (fd < 0) throw std::runtime_error("tls: cannot create " + tmp);
  FILE* f = ::fdopen(fd, "wb");
  if (!f) {
    ::close(fd);
    throw std::runtime_error("tls: cannot open " + tmp);
  }
  return f;
}

void commit_tmp(FILE* f, const std::string& tmp, const std::string& path) {
  fflush(f);
  ::fsync(fileno(f));
  fclose(f);
  if (::rename(tmp.c_str(), path.c_str()) != 0) {
    ::unlink(tmp.c_str());
    throw std::runtime_error("tls: cannot install " + path);
  }
}

void write_pem_key(const std::string& path, EVP_PKEY* k) {
  std::string tmp;
  FILE* f = open_private_tmp(path, 0600, tmp);
  PEM_write_PrivateKey(f, k, nullptr, nullptr, 0, nullptr, nullptr);
  commit_tmp(f, tmp, path);
}

void write_pem_cert(const std::string& path, X509* c) {
  std::string tmp;
  FILE* f = open_private_tmp(path, 0644, tmp);
  PEM_write_X509(f, c);
  commit_tmp(f, tmp, path);
}

// exclusive advisory lock on <dir>/.lock for the lifetime of the object: services started
// together by aios-init serialise their "generate if missing" so exactly one CA is created
struct DirLock {
  int fd = -1;
  explicit DirLock(const std::string& dir) {
    fd = ::open((dir + "/.lock").c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (fd >= 0) ::flock(fd, LOCK_EX);
  }
  ~DirLock() {
    if (fd >= 0) {
      ::flock(fd, LOCK_UN);
      ::close(fd);
    }
  }
};

X509Ptr read_cert(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return X509Ptr();
  X509* c = PEM_read_X509(f, nullptr, nullptr, nullptr);
  fclose(f);
  return X509Ptr(c);
}

PkeyPtr read_key(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return PkeyPtr();
  EVP_PKEY* k = PEM_read_PrivateKey(f, nullptr, nullptr, nullptr);
  fclose(f);
  return PkeyPtr(k);
}

}  // namespace

Json TlsManager::paths() const {
  return Json::object({{"ca_cert", dir_ + "/ca.crt"}, {"ca_key", dir_ + "/ca.key"},
                       {"server_cert", dir_ + "/server.crt"}, {"server_key", dir_ + "/server.key"}});
}

bool TlsManager::certs_exist() const {
  return file_exists(dir_ + "/ca.crt") && file_exists(dir_ + "/server.crt") && file_exists(dir_ + "/server.key");
}

Json TlsManager::generate_self_signed(const std::string& service, int days) {
  Json p = paths();
  if (certs_exist()) {
    p.set("generated", false);
    return p;
  }
  mkdirs(dir_);
  DirLock lock(dir_);
  if (certs_exist()) {  // another service generated them while we waited for the lock
    p.set("generated", false);
    return p;
  }
  PkeyPtr ca_key = ec_key();
  X509Ptr ca = make_cert(ca_key.get(), "aiOS Root CA", nullptr, nullptr, 3650, true, "");
  PkeyPtr srv_key = ec_key();
  const std::string san = "DNS:localhost,IP:127.0.0.1" + (service.empty() ? std::string() : ",DNS:" + service);
  X509Ptr srv = make_cert(srv_key.get(), service.empty() ? "localhost" : service, ca.get(), ca_key.get(), days, false, san);
  write_pem_key(dir_ + "/ca.key", ca_key.get());
  write_pem_cert(dir_ + "/ca.crt", ca.get());
  write_pem_key(dir_ + "/server.key", srv_key.get());
  write_pem_cert(dir_ + "/server.crt", srv.get());
  p.set("generated", true);
  return p;
}

Json TlsManager::verify() const {
  Json r = Json::object({{"exists", certs_exist()}});
  X509Ptr ca = read_cert(dir_ + "/ca.crt"), srv = read_cert(dir_ + "/server.crt");
  PkeyPtr key = read_key(dir_ + "/server.key");
  const bool parsed = ca && srv && key;
  r.set("parsed", parsed);
  bool signed_ok = false, in_window = false, key_match = false;
  if (parsed) {
    EVP_PKEY* ca_pub = X509_get0_pubkey(ca.get());
    signed_ok = X509_verify(srv.get(), ca_pub) == 1;
    in_window = X509_cmp_current_time(X509_get0_notBefore(srv.get())) < 0 &&
                X509_cmp_current_time(X509_get0_notAfter(srv.get())) > 0;
    key_match = X509_check_private_key(srv.get(), key.get()) == 1;
  }
  r.set("signed_by_ca", signed_ok);
  r.set("valid_now", in_window);
  r.set("key_matches", key_match);
  r.set("ok", parsed && signed_ok && in_window && key_match);
  return r;
}

}  // namespace aiosn
