// Planner heuristics + LLM-output parsing + reactive-tier heuristic executor.
// Reference behaviour: agent-core/src/task_planner.rs:143-676 and autonomy.rs:1149-2375.
#include <algorithm>
#include <functional>
#include <cctype>
#include <set>

#include "orchestrator.h"

namespace aiosn {

namespace {

bool has_word(const std::string& text, const std::string& word) {
  std::string w;
  for (size_t i = 0; i <= text.size(); ++i) {
    const char c = i < text.size() ? text[i] : ' ';
    if (std::isalnum((unsigned char)c) || c == '_') {
      w += c;
    } else {
      if (w == word) return true;
      w.clear();
    }
  }
  return false;
}

Json make_task(const std::string& goal_id, const std::string& desc, const std::string& level,
               const std::vector<std::string>& tools, const std::string& dep) {
  Json t = Json::object();
  t.set("id", uuid4());
  t.set("goal_id", goal_id);
  t.set("description", desc);
  t.set("assigned_agent", "");
  t.set("status", "pending");
  t.set("intelligence_level", level);
  Json tl = Json::array();
  for (auto& x : tools) tl.push(x);
  t.set("required_tools", tl);
  Json deps = Json::array();
  if (!dep.empty()) deps.push(dep);
  t.set("depends_on", deps);
  t.set("input_json", "");
  t.set("output_json", "");
  t.set("created_at", now_unix());
  t.set("started_at", 0);
  t.set("completed_at", 0);
  t.set("error", "");
  return t;
}

std::string trim_chars(const std::string& s, const std::function<bool(char)>& keep) {
  size_t a = 0, b = s.size();
  while (a < b && !keep(s[a])) ++a;
  while (b > a && !keep(s[b - 1])) --b;
  return s.substr(a, b - a);
}

}  // namespace

// =============================================================================== planner
namespace planner {

const char* kDecomposeSystemPrompt =
    "You are aiOS task planner. Decompose goals into executable steps. Respond with ONLY valid JSON.";

std::string ai_decomposition_prompt(const std::string& description) {
  return "Decompose this goal into 2-5 concrete steps that can be executed with system tools.\nGoal: " + description +
         "\n\nAvailable tool namespaces: fs, process, service, net, firewall, pkg, sec, monitor, web, git, code, "
         "plugin, container, email\n\nRespond with ONLY a JSON array:\n"
         "[{\"description\": \"step description\", \"tools\": [\"namespace\"]}]";
}

std::string classify(const std::string& description) {
  const std::string d = lower(description);
  if (contains(d, "status") || contains(d, "health") || contains(d, "uptime") || contains(d, "ping")) return "reactive";
  if ((contains(d, "email") || contains(d, "mail")) && (contains(d, "send") || contains(d, "@"))) return "reactive";
  if (contains(d, "call ") || contains(d, "execute ") || contains(d, "run ")) {
    for (const char* p : {"fs.", "process.", "service.", "net.", "monitor.", "email.", "pkg.", "sec."})
      if (contains(d, p)) return "reactive";
  }
  if (contains(d, "analyze") || contains(d, "plan") || contains(d, "design") || contains(d, "security audit") ||
      contains(d, "architecture"))
    return "strategic";
  if (contains(d, "read file") || contains(d, "list") || contains(d, "check disk") || contains(d, "log"))
    return "operational";
  return "tactical";
}

std::vector<std::string> infer_tools(const std::string& description) {
  const std::string d = lower(description);
  std::vector<std::string> t;
  if (contains(d, "file") || has_word(d, "read") || has_word(d, "write") || contains(d, "directory") ||
      contains(d, "disk"))
    t.push_back("fs");
  if (contains(d, "process") || has_word(d, "kill") || has_word(d, "spawn")) t.push_back("process");
  if (has_word(d, "service") || has_word(d, "restart") || has_word(d, "systemctl")) t.push_back("service");
  if (contains(d, "network") || contains(d, "firewall") || has_word(d, "dns") || has_word(d, "ping"))
    t.push_back("net");
  if (has_word(d, "install") || has_word(d, "package") || has_word(d, "apt")) t.push_back("pkg");
  if (contains(d, "security") || contains(d, "permission") || has_word(d, "audit") || contains(d, "vulnerab"))
    t.push_back("sec");
  if (contains(d, "plugin") || contains(d, "script")) t.push_back("plugin");
  if (contains(d, "email") || contains(d, "smtp") || contains(d, "mail") || contains(d, "newsletter"))
    t.push_back("email");
  if (contains(d, "monitor") || has_word(d, "cpu") || has_word(d, "memory") || contains(d, "metric"))
    t.push_back("monitor");
  if (contains(d, "container") || contains(d, "podman") || contains(d, "docker")) t.push_back("container");
  return t;
}

std::string extract_service_name(const std::string& d) {
  for (const char* s : {"nginx", "apache", "postgres", "mysql", "redis", "docker", "ssh", "systemd", "cron",
                        "mongodb", "elasticsearch"})
    if (contains(d, s)) return s;
  return "the service";
}

std::vector<std::pair<std::string, std::vector<std::string>>> analyze_steps(const std::string& description) {
  const std::string d = lower(description);
  std::vector<std::pair<std::string, std::vector<std::string>>> s;
  if (contains(d, "restart") || contains(d, "deploy")) {
    const std::string svc = extract_service_name(d);
    s.push_back({"Check current status of " + svc, {"service", "monitor"}});
    s.push_back({"Stop " + svc + " gracefully", {"service"}});
    s.push_back({"Start " + svc + " and verify", {"service", "monitor"}});
  } else if (contains(d, "security") || contains(d, "audit")) {
    s.push_back({"Gather system security configuration", {"sec", "fs"}});
    s.push_back({"Analyze security posture and vulnerabilities", {"sec"}});
    s.push_back({"Generate security report with recommendations", {"fs"}});
  } else if (contains(d, "install") || contains(d, "setup")) {
    s.push_back({"Check prerequisites for: " + description, {"pkg", "fs"}});
    s.push_back({"Install: " + description, {"pkg"}});
    s.push_back({"Verify installation and configure", {"service", "fs"}});
  } else if (contains(d, "network") || contains(d, "connectivity")) {
    s.push_back({"Check network interfaces and routing", {"net"}});
    s.push_back({"Test DNS resolution and connectivity", {"net"}});
    s.push_back({"Diagnose and apply fixes", {"net", "firewall"}});
  }
  return s;
}

Json decompose(const std::string& goal_id, const std::string& description, const std::string& level) {
  Json out = Json::array();
  if (level == "reactive" || level == "operational") {
    out.push(make_task(goal_id, description, level, infer_tools(description), ""));
    return out;
  }
  // keyword multi-step fallback for tactical / strategic (the AI path is tried first by the service)
  std::string prev;
  int i = 0;
  for (auto& st : analyze_steps(description)) {
    Json t = make_task(goal_id, st.first, i == 0 ? "operational" : level, st.second, prev);
    prev = t.get_str("id");
    out.push(t);
    ++i;
  }
  if (!out.size()) out.push(make_task(goal_id, description, level, infer_tools(description), ""));
  return out;
}

Json parse_ai_decomposition(const std::string& text, const std::string& goal_id, const std::string& level) {
  const std::string cleaned = trim(llm::strip_think(text));
  Json arr;
  if (!(Json::try_parse(cleaned, arr) && arr.is_arr())) {
    arr = Json();
    const auto fence = cleaned.find("```");
    if (fence != std::string::npos) {
      std::string after = cleaned.substr(fence + 3);
      const auto nl = after.find('\n');
      after = nl == std::string::npos ? after : after.substr(nl + 1);
      const auto end = after.find("```");
      if (end != std::string::npos) Json::try_parse(trim(after.substr(0, end)), arr);
    } else {
      const auto b = cleaned.find('['), e = cleaned.rfind(']');
      if (b != std::string::npos && e != std::string::npos && e > b) Json::try_parse(cleaned.substr(b, e - b + 1), arr);
    }
    if (!arr.is_arr()) {
      // an object wrapping the list ({"steps": [...]}) is accepted too
      Json obj;
      if (llm::extract_json(cleaned, obj))
        for (const char* k : {"steps", "tasks", "plan"})
          if (obj[k].is_arr()) {
            arr = obj[k];
            break;
          }
    }
  }
  Json out = Json::array();
  if (!arr.is_arr() || arr.size() == 0 || arr.size() > 10) return out;
  std::string prev;
  int i = 0;
  for (auto& step : arr.as_arr()) {
    std::string desc = step.is_str() ? step.as_str() : step.get_str("description");
    if (desc.empty()) desc = step.get_str("step", step.get_str("task"));
    if (desc.empty()) continue;
    std::vector<std::string> tools;
    for (auto& tl : step["tools"].as_arr())
      if (tl.is_str()) tools.push_back(tl.as_str());
    Json t = make_task(goal_id, desc, i == 0 ? "operational" : level, tools, prev);
    prev = t.get_str("id");
    out.push(t);
    ++i;
  }
  return out;
}

}  // namespace planner

// =============================================================================== llm
namespace llm {

std::string strip_think(const std::string& text) {
  std::string r = text;
  while (true) {
    const auto s = r.find("<think>");
    if (s == std::string::npos) break;
    const auto e = r.find("</think>", s);
    if (e == std::string::npos) {
      r = r.substr(0, s);
      break;
    }
    r = r.substr(0, s) + r.substr(e + 8);
  }
  return r;
}

bool extract_json(const std::string& text, Json& out) {
  const std::string t = trim(strip_think(trim(text)));
  if (Json::try_parse(t, out)) return true;
  const auto fence = t.find("```");
  if (fence != std::string::npos) {
    std::string after = t.substr(fence + 3);
    const auto nl = after.find('\n');
    after = nl == std::string::npos ? after : after.substr(nl + 1);
    const auto end = after.find("```");
    if (end != std::string::npos && Json::try_parse(trim(after.substr(0, end)), out)) return true;
  }
  // first balanced {...} (string-aware, unlike the reference's plain brace counter)
  const auto start = t.find('{');
  if (start != std::string::npos) {
    int depth = 0;
    bool in_str = false, esc = false;
    for (size_t i = start; i < t.size(); ++i) {
      const char c = t[i];
      if (in_str) {
        if (esc) esc = false;
        else if (c == '\\') esc = true;
        else if (c == '"') in_str = false;
        continue;
      }
      if (c == '"') in_str = true;
      else if (c == '{') ++depth;
      else if (c == '}' && --depth == 0) {
        if (Json::try_parse(t.substr(start, i - start + 1), out)) return true;
        break;
      }
    }
  }
  return false;
}

namespace {
const char* kNamespaces[] = {"fs", "process", "service", "net", "firewall", "pkg", "sec", "monitor",
                             "hw", "web", "git", "code", "self", "plugin", "container", "email"};

bool tool_name_at(const std::string& s, size_t pos, std::string& name) {
  size_t i = pos;
  while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '.')) ++i;
  std::string cand = s.substr(pos, i - pos);
  while (!cand.empty() && cand.back() == '.') cand.pop_back();
  const auto dot = cand.find('.');
  if (dot == std::string::npos || dot == 0 || dot + 1 >= cand.size()) return false;
  const std::string ns = cand.substr(0, dot);
  for (auto* k : kNamespaces)
    if (ns == k) {
      name = cand;
      return true;
    }
  return false;
}

Json call(const std::string& tool, const Json& input) {
  return Json::object({{"tool", tool}, {"input", input.is_obj() ? input : Json::object()}});
}

std::map<std::string, Json> find_tool_parameters(const Json& p) {
  std::map<std::string, Json> params;
  if (!p.is_obj()) return params;
  for (const char* k : {"parameters", "inputs", "arguments", "input", "params", "tool_input"}) {
    const Json& v = p[k];
    if (!v.is_obj()) continue;
    const std::string tn = v.get_str("tool");
    if (!tn.empty()) {
      Json clean = Json::object();
      for (auto& kv : v.as_obj())
        if (kv.first != "tool") clean.set(kv.first, kv.second);
      params[tn] = clean;
    } else {
      params["*"] = v;
    }
  }
  for (auto& item : p["tool_calls"].as_arr()) {
    std::string n = item.get_str("tool", item.get_str("name", item.get_str("function")));
    for (const char* k : {"input", "parameters", "params", "arguments"})
      if (!n.empty() && item.has(k)) {
        params[n] = item[k];
        break;
      }
  }
  auto w = params.find("*");
  if (w != params.end()) {
    Json wild = w->second;
    params.erase(w);
    for (auto& t : p["tools_needed"].as_arr())
      if (t.is_str() && !params.count(t.as_str())) params[t.as_str()] = wild;
  }
  return params;
}

Json first_of(const Json& o, std::initializer_list<const char*> keys) {
  for (auto* k : keys)
    if (o.has(k)) return o[k];
  return Json::object();
}
}  // namespace

Json tools_from_natural_language(const std::string& text) {
  Json calls = Json::array();
  std::set<std::string> seen;
  for (const char* trig : {"call ", "Call ", "use ", "Use ", "execute ", "Execute ", "run ", "Run "}) {
    size_t pos = 0;
    while ((pos = text.find(trig, pos)) != std::string::npos) {
      pos += std::string(trig).size();
      std::string n;
      if (tool_name_at(text, pos, n) && seen.insert(n).second) calls.push(call(n, Json::object()));
    }
  }
  if (!calls.size()) {
    for (auto* ns : kNamespaces) {
      const std::string pre = std::string(ns) + ".";
      size_t pos = 0;
      while ((pos = text.find(pre, pos)) != std::string::npos) {
        const bool boundary = pos == 0 || !std::isalnum((unsigned char)text[pos - 1]);
        std::string n;
        if (boundary && tool_name_at(text, pos, n) && seen.insert(n).second) calls.push(call(n, Json::object()));
        pos += pre.size();
      }
    }
  }
  return calls;
}

Json parse_tool_calls(const std::string& text) {
  Json calls = Json::array();
  Json p;
  if (!extract_json(text, p)) return tools_from_natural_language(text);
  if (p.is_arr()) {  // a bare list of calls
    for (auto& tc : p.as_arr()) {
      const std::string n = tc.get_str("tool", tc.get_str("name"));
      if (!n.empty()) calls.push(call(n, first_of(tc, {"input", "parameters", "params", "arguments"})));
    }
    return calls;
  }
  if (p["tool_calls"].is_arr()) {
    for (auto& tc : p["tool_calls"].as_arr()) {
      const std::string n = tc.get_str("tool", tc.get_str("name"));
      if (!n.empty()) calls.push(call(n, first_of(tc, {"input", "parameters", "params", "arguments"})));
    }
  } else {
    auto extra = find_tool_parameters(p);
    for (auto& step : p["steps"].as_arr()) {
      std::string n = step.get_str("tool", step.get_str("action", step.get_str("name")));
      if (!n.empty() && n.find('.') != std::string::npos) {
        calls.push(call(n, first_of(step, {"input", "parameters", "params", "arguments", "args"})));
      } else {
        const std::string t = step.is_str() ? step.as_str() : step.get_str("task", step.get_str("description"));
        const Json nl = tools_from_natural_language(t);
        for (auto& c : nl.as_arr()) calls.push(c);
      }
    }
    if (!calls.size())
      for (auto& t : p["tools_needed"].as_arr()) {
        if (t.is_obj()) {
          const std::string n = t.get_str("tool", t.get_str("name"));
          if (!n.empty()) calls.push(call(n, first_of(t, {"input", "parameters"})));
        } else if (t.is_str()) {
          calls.push(call(t.as_str(), extra.count(t.as_str()) ? extra[t.as_str()] : Json::object()));
        }
      }
    if (!calls.size())
      for (auto& a : p["actions"].as_arr()) {
        const std::string n = a.get_str("tool", a.get_str("name"));
        if (!n.empty()) calls.push(call(n, first_of(a, {"input", "parameters", "params"})));
      }
    // enrich empty inputs from parameters found elsewhere in the response
    Json enriched = Json::array();
    for (auto& c : calls.as_arr()) {
      Json cc = c;
      if (c["input"].size() == 0 && extra.count(c.get_str("tool"))) cc.set("input", extra[c.get_str("tool")]);
      enriched.push(cc);
    }
    calls = enriched;
  }
  if (!calls.size()) return tools_from_natural_language(text);
  return calls;
}

bool parse_clarification(const std::string& text, std::string& q) {
  Json p;
  if (!extract_json(text, p) || !p.get_bool("needs_clarification")) return false;
  std::string out;
  int i = 0;
  for (auto& x : p["questions"].as_arr())
    if (x.is_str()) out += (out.empty() ? "" : "\n") + std::to_string(++i) + ". " + x.as_str();
  if (out.empty()) out = p.get_str("reasoning", "I need more information to proceed with this task.");
  q = out;
  return true;
}

bool is_done_signal(const std::string& text) {
  Json p;
  return extract_json(text, p) && p.is_obj() && p.get_bool("done");
}

namespace {
std::string extract_quoted_field(const std::string& text, std::initializer_list<const char*> prefixes) {
  const std::string tl = lower(text);
  for (auto* pre : prefixes) {
    const std::string pl = lower(pre);
    const auto pos = tl.find(pl);
    if (pos == std::string::npos) continue;
    std::string after = text.substr(pos + pl.size());
    size_t a = 0;
    while (a < after.size() && std::isspace((unsigned char)after[a])) ++a;
    after = after.substr(a);
    if (!after.empty() && (after[0] == '\'' || after[0] == '"')) {
      const auto end = after.find(after[0], 1);
      if (end != std::string::npos && end > 1) return after.substr(1, end - 1);
    }
    size_t end_pos = after.size();
    const std::string al = lower(after);
    for (const char* term : {" body:", " body ", " message:", " subject:", " \xE2\x80\x94 ", " with ", " and body"}) {
      const auto p = al.find(term);
      if (p != std::string::npos && p > 0 && p < end_pos) end_pos = p;
    }
    const std::string v = trim(after.substr(0, end_pos));
    if (!v.empty()) return v;
  }
  return "";
}

bool extract_email(const std::string& desc, Json& out) {
  const auto b = desc.find('{');
  if (b != std::string::npos) {
    Json j;
    if (extract_json(desc.substr(b), j) && j.has("to")) {
      out = j;
      return true;
    }
  }
  std::string to;
  for (auto& w : split_ws(desc)) {
    const std::string c = trim_chars(w, [](char ch) {
      return std::isalnum((unsigned char)ch) || ch == '@' || ch == '.' || ch == '_' || ch == '-' || ch == '+';
    });
    if (c.find('@') != std::string::npos && c.find('.') != std::string::npos && c.size() >= 5) {
      to = c;
      break;
    }
  }
  if (to.empty()) return false;
  std::string subject = extract_quoted_field(desc, {"subject:", "subject ", "subject="});
  std::string body = extract_quoted_field(desc, {"body:", "body ", "body=", "message:"});
  if (subject.empty()) {
    std::string w = desc;
    const auto p = w.find(to);
    if (p != std::string::npos) w.erase(p, to.size());
    w = trim_chars(trim(w), [](char ch) { return std::isalnum((unsigned char)ch); });
    subject = (!w.empty() && w.size() < 200) ? w : "Message from aiOS";
  }
  if (body.empty()) body = subject;
  out = Json::object({{"to", to}, {"subject", subject}, {"body", body}});
  return true;
}

bool extract_host(const std::string& text, std::string& host) {
  auto words = split_ws(text);
  auto clean = [](const std::string& w) {
    return trim_chars(w, [](char c) { return std::isalnum((unsigned char)c) || c == '.' || c == ':' || c == '-'; });
  };
  for (size_t i = 0; i + 1 < words.size(); ++i) {
    if (words[i] == "ping" || words[i] == "net.ping" || words[i] == "resolve" || words[i] == "lookup") {
      const std::string n = clean(words[i + 1]);
      if (n.find('.') != std::string::npos || n.find(':') != std::string::npos) {
        host = n;
        return true;
      }
    }
  }
  for (auto& w : words) {
    const std::string c = clean(w);
    if (c.find('.') != std::string::npos && c.size() >= 4 && std::isalnum((unsigned char)c[0]) &&
        c.find("net.") != 0 && c.find("monitor.") != 0) {
      host = c;
      return true;
    }
  }
  return false;
}

bool extract_path(const std::string& desc, std::string& path) {
  for (auto& w : split_ws(desc)) {
    const std::string c = trim_chars(w, [](char ch) { return ch != '\'' && ch != '"' && ch != '`'; });
    if (c.size() >= 2 && c[0] == '/') {
      path = c;
      while (!path.empty() && (path.back() == ',' || path.back() == '.' || path.back() == ';')) path.pop_back();
      return true;
    }
  }
  return false;
}

bool extract_service(const std::string& text, std::string& svc) {
  for (const char* s : {"aios-orchestrator", "aios-api-gateway", "aios-runtime", "aios-tools", "aios-memory", "nginx",
                        "apache", "postgres", "mysql", "redis", "docker", "sshd", "ssh", "cron", "mongodb",
                        "elasticsearch", "podman"})
    if (contains(text, s)) {
      svc = s;
      return true;
    }
  return false;
}
}  // namespace

bool explicit_tool_call(const std::string& desc, Json& out) {
  // "call fs.read with {...}" / "fs.read {...}"
  for (auto* ns : kNamespaces) {
    const std::string pre = std::string(ns) + ".";
    size_t pos = 0;
    while ((pos = desc.find(pre, pos)) != std::string::npos) {
      std::string n;
      if ((pos == 0 || !std::isalnum((unsigned char)desc[pos - 1])) && tool_name_at(desc, pos, n)) {
        Json input = Json::object();
        const auto b = desc.find('{', pos);
        if (b != std::string::npos) {
          Json j;
          if (extract_json(desc.substr(b), j) && j.is_obj()) input = j;
        }
        out = call(n, input);
        return true;
      }
      pos += pre.size();
    }
  }
  return false;
}

Json heuristic_calls(const Json& task) {
  // reactive tier: map task text to tool calls without an LLM (autonomy.rs:1149-1249)
  const std::string desc = task.get_str("description"), d = lower(desc);
  bool email_tool = false;
  for (auto& t : task["required_tools"].as_arr())
    if (t.as_str() == "email") email_tool = true;
  Json out = Json::array();
  const bool is_email = email_tool || contains(d, "email.send") ||
                        ((contains(d, "email") || contains(d, "mail")) && (contains(d, "send") || contains(d, "@")));
  Json in;
  if (is_email && extract_email(desc, in)) {
    out.push(call("email.send", in));
    return out;
  }
  if (contains(d, "monitor.cpu") || (contains(d, "cpu") && contains(d, "usage"))) {
    out.push(call("monitor.cpu", Json::object()));
    return out;
  }
  if (contains(d, "monitor.memory") || (contains(d, "memory") && contains(d, "usage"))) {
    out.push(call("monitor.memory", Json::object()));
    return out;
  }
  if (contains(d, "monitor.disk") || (contains(d, "disk") && (contains(d, "usage") || contains(d, "space")))) {
    out.push(call("monitor.disk", Json::object()));
    return out;
  }
  std::string host;
  if ((contains(d, "ping ") || contains(d, "net.ping")) && extract_host(d, host)) {
    out.push(call("net.ping", Json::object({{"host", host}})));
    return out;
  }
  if (contains(d, "dns") && (contains(d, "lookup") || contains(d, "resolve")) && extract_host(d, host)) {
    out.push(call("net.dns", Json::object({{"host", host}, {"hostname", host}})));
    return out;
  }
  std::string path;
  if ((contains(d, "read") || contains(d, "cat") || contains(d, "fs.read")) && extract_path(desc, path)) {
    out.push(call("fs.read", Json::object({{"path", path}})));
    return out;
  }
  std::string svc;
  if ((contains(d, "service") || contains(d, "systemctl")) && contains(d, "status") && extract_service(d, svc)) {
    out.push(call("service.status", Json::object({{"name", svc}})));
    return out;
  }
  Json ex;
  if (explicit_tool_call(desc, ex)) out.push(ex);
  return out;
}

std::string json_to_readable(const Json& v, int depth) {
  const std::string pad((size_t)depth * 2, ' ');
  switch (v.type()) {
    case Json::NUL: return "none";
    case Json::BOOL: return v.as_bool() ? "yes" : "no";
    case Json::NUM: return v.dump();
    case Json::STR: return v.as_str();
    case Json::ARR: {
      if (!v.size()) return "(empty)";
      std::string out;
      size_t i = 0;
      for (auto& x : v.as_arr()) {
        if (i++ >= 20) {
          out += pad + "- ... (" + std::to_string(v.size() - 20) + " more)\n";
          break;
        }
        out += pad + "- " + (x.is_obj() || x.is_arr() ? "\n" + json_to_readable(x, depth + 1) : json_to_readable(x)) + "\n";
      }
      return out;
    }
    case Json::OBJ: {
      std::string out;
      for (auto& kv : v.as_obj()) {
        std::string key = kv.first;
        std::replace(key.begin(), key.end(), '_', ' ');
        if (kv.second.is_obj() || kv.second.is_arr())
          out += pad + key + ":\n" + json_to_readable(kv.second, depth + 1) + "\n";
        else
          out += pad + key + ": " + json_to_readable(kv.second) + "\n";
      }
      return out;
    }
  }
  return "";
}

std::string summarize_tool_output(const std::string& tool, const Json& output, size_t max_chars) {
  std::string s;
  if (tool == "fs.read" && output.has("content")) {
    const std::string c = output.get_str("content");
    s = "Read " + output.get_str("size", std::to_string(c.size())) + " bytes:\n" + c;
  } else if (tool == "fs.list" && output["entries"].is_arr()) {
    s = std::to_string(output["entries"].size()) + " entries: ";
    size_t i = 0;
    for (auto& e : output["entries"].as_arr()) {
      if (i++ >= 50) break;
      s += e.get_str("name") + (e.get_str("type") == "directory" ? "/" : "") + " ";
    }
  } else if (tool == "process.list" && output["processes"].is_arr()) {
    s = std::to_string(output["processes"].size()) + " processes";
  } else {
    s = json_to_readable(output);
  }
  if (s.size() > max_chars) s = s.substr(0, max_chars) + "... (truncated)";
  return s;
}

}  // namespace llm

}  // namespace aiosn
