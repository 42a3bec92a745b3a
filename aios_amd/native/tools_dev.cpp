// web (5), git (10), code (2), self (4), plugin (5), container (6) and email (1) tools.
// Reference: tools/src/{web,git,code,self_update,plugin,container,email}/*.rs.
#include <dirent.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <openssl/hmac.h>
#include <sys/socket.h>
#include <sys/statvfs.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <regex>
#include <set>

#include "tools.h"

namespace aiosn {

namespace {

void add(std::vector<ToolSpec>& v, const char* name, const char* desc, std::vector<std::string> reg_caps,
         const char* risk, bool idem, bool rev, int timeout, std::vector<std::string> caps, ToolHandler fn) {
  ToolSpec s;
  s.def.name = name;
  s.def.ns = std::string(name).substr(0, std::string(name).find('.'));
  s.def.description = desc;
  s.def.required_caps = std::move(reg_caps);
  s.def.risk_level = risk;
  s.def.idempotent = idem;
  s.def.reversible = rev;
  s.def.timeout_ms = timeout;
  s.caps = std::move(caps);
  s.fn = std::move(fn);
  v.push_back(std::move(s));
}

CmdResult sh(const std::vector<std::string>& argv, int timeout_ms = 30000, const std::string& cwd = "",
             const std::string& stdin_data = "") {
  CmdLimits l;
  l.timeout_ms = timeout_ms;
  l.cwd = cwd;
  l.stdin_data = stdin_data;
  return run_cmd(argv, l);
}

std::string http_url(const Json& in, const char* key = "url") {
  const std::string u = req_str(in, key);
  if (!starts_with(u, "http://") && !starts_with(u, "https://")) tool_fail("url must start with http:// or https://");
  return u;
}

struct HttpResp {
  int status = 0;
  std::string body, err;
  bool ok = false;
};

HttpResp curl_req(const std::string& method, const std::string& url, const Json& headers, const std::string& body,
                  const std::string& bearer, int timeout_s, bool follow) {
  std::vector<std::string> a{"curl", "-sS", "-X", method, "--max-time", std::to_string(std::max(1, timeout_s)),
                             "-w", "\n%{http_code}"};
  if (follow) a.push_back("-L");
  for (auto& kv : headers.as_obj()) {
    a.push_back("-H");
    a.push_back(kv.first + ": " + kv.second.str_or(kv.second.dump()));
  }
  if (!bearer.empty()) {
    a.push_back("-H");
    a.push_back("Authorization: Bearer " + bearer);
  }
  if (!body.empty()) {
    a.push_back("--data-binary");
    a.push_back("@-");
  }
  a.push_back(url);
  CmdResult r = sh(a, timeout_s * 1000 + 5000, "", body);
  HttpResp h;
  if (r.exit_code != 0) {
    h.err = trim(r.err.empty() ? "curl exit " + std::to_string(r.exit_code) : r.err);
    return h;
  }
  const auto nl = r.out.rfind('\n');
  h.status = nl == std::string::npos ? 0 : std::atoi(r.out.c_str() + nl + 1);
  h.body = nl == std::string::npos ? "" : r.out.substr(0, nl);
  h.ok = h.status >= 200 && h.status < 400;
  return h;
}

std::string strip_html(const std::string& html) {
  std::string s = std::regex_replace(html, std::regex("<(script|style)[^>]*>[\\s\\S]*?</\\1>", std::regex::icase), " ");
  s = std::regex_replace(s, std::regex("<[^>]+>"), " ");
  static const std::pair<const char*, const char*> ents[] = {
      {"&amp;", "&"}, {"&lt;", "<"}, {"&gt;", ">"}, {"&quot;", "\""}, {"&#39;", "'"}, {"&nbsp;", " "}};
  for (auto& e : ents) s = std::regex_replace(s, std::regex(e.first), e.second);
  s = std::regex_replace(s, std::regex("[ \\t\\r\\n]+"), " ");
  return trim(s);
}

// ------------------------------------------------------------------------------ git
std::string repo(const Json& in) {
  const std::string p = in.has("repo_path") ? abs_path(in, "repo_path") : abs_path(in, "path");
  return p;
}
CmdResult git(const std::string& repo_path, std::vector<std::string> args, int timeout_ms = 30000) {
  if (!have_cmd("git")) tool_fail("git not available");
  std::vector<std::string> a{"git", "-C", repo_path};
  a.insert(a.end(), args.begin(), args.end());
  return sh(a, timeout_ms);
}
CmdResult git_ok(const std::string& repo_path, std::vector<std::string> args, int timeout_ms = 30000) {
  CmdResult r = git(repo_path, args, timeout_ms);
  if (r.exit_code != 0) tool_fail("git " + (args.empty() ? "" : args[0]) + " failed: " + trim(r.err + r.out));
  return r;
}
std::string valid_ref(const std::string& s) {
  static const std::regex re("^[A-Za-z0-9._/-]{1,200}$");
  if (!std::regex_match(s, re) || starts_with(s, "-")) tool_fail("invalid ref/remote name: " + s);
  return s;
}

// ------------------------------------------------------------------------------ plugins
const char* kDangerous[][3] = {
    {"os.system(", "30", "Arbitrary command execution via os.system"},
    {"subprocess.call(", "20", "Subprocess execution"},
    {"subprocess.Popen(", "20", "Subprocess execution"},
    {"subprocess.run(", "15", "Subprocess execution"},
    {"eval(", "25", "Dynamic code evaluation"},
    {"exec(", "25", "Dynamic code execution"},
    {"compile(", "15", "Dynamic code compilation"},
    {"__import__(", "20", "Dynamic module import"},
    {"importlib.import_module(", "15", "Dynamic module import"},
    {"open(", "5", "File access (check paths)"},
    {"shutil.rmtree(", "20", "Recursive directory deletion"},
    {"os.remove(", "10", "File deletion"},
    {"os.unlink(", "10", "File deletion"},
    {"os.rmdir(", "10", "Directory deletion"},
    {"socket.socket(", "10", "Raw socket creation"},
    {"ctypes.", "20", "C library access"},
    {"os.chmod(", "10", "Permission modification"},
    {"os.chown(", "10", "Ownership modification"},
    {"os.setuid(", "30", "Privilege escalation"},
    {"os.setgid(", "30", "Privilege escalation"},
};

std::string valid_plugin_name(const std::string& n) {
  static const std::regex re("^[a-z][a-z0-9_]{0,63}$");
  std::string s = starts_with(n, "plugin.") ? n.substr(7) : n;
  if (!std::regex_match(s, re)) tool_fail("plugin name must match [a-z][a-z0-9_]*: " + n);
  return s;
}

Json write_plugin(ToolContext& ctx, const std::string& name, const std::string& desc, const std::string& code,
                  const Json& caps, const Json& deps, const Json& next, const std::string& mode) {
  Json val = plugin_validate(code);
  if (!val.get_bool("safe"))
    tool_fail("Plugin code rejected: risk_score=" + std::to_string(val.get_int("risk_score")) + ", findings: " +
              val["findings"].dump());
  if (code.find("def main(") == std::string::npos) tool_fail("plugin code must define main(input_data) -> dict");
  const std::string dir = ctx.paths->plugin_dir();
  mkdirs(dir);
  const std::string script = dir + "/" + name + ".py", meta_path = dir + "/" + name + ".meta.json";
  {
    std::ofstream f(script);
    f << plugin_wrapper(code);
    if (!f) tool_fail("cannot write " + script);
  }
  Json meta = Json::object();
  meta.set("tool_name", "plugin." + name);
  meta.set("description", desc);
  meta.set("capabilities", caps.is_arr() ? caps : Json::array());
  meta.set("dependencies", deps.is_arr() ? deps : Json::array());
  meta.set("author", "aios");
  meta.set("created_at", now_rfc3339());
  meta.set("timeout_ms", 30000);
  meta.set("next_plugins", next.is_arr() ? next : Json::array());
  meta.set("output_mode", mode.empty() ? "pipe" : mode);
  meta.set("validation", val);
  std::ofstream m(meta_path);
  m << meta.dump(2);
  return Json::object({{"script_path", script}, {"metadata_path", meta_path}});
}

Json pip_install(const Json& pkgs) {
  Json installed = Json::array();
  std::string err;
  for (auto& p : pkgs.as_arr()) {
    static const std::regex re("^[A-Za-z0-9][A-Za-z0-9._-]*([<>=!~]=?[A-Za-z0-9.*]+)?$");
    if (!std::regex_match(p.as_str(), re)) {
      err += "invalid package " + p.as_str() + "; ";
      continue;
    }
    SandboxLimits lim;
    lim.allow_network = true;
    lim.timeout_ms = 55000;
    lim.cpu_seconds = 55;
    lim.mem_bytes = 1ull << 30;
    SandboxResult r = sandbox_exec("pip3", {"install", "--user", "--quiet", p.as_str()}, "", lim);
    if (r.success) installed.push(p);
    else err += p.as_str() + ": " + trim(r.error).substr(0, 300) + "; ";
  }
  return Json::object({{"installed", installed}, {"error", err}});
}

const std::map<std::string, std::pair<std::string, std::string>>& templates() {
  // name -> (description, code)
  static const std::map<std::string, std::pair<std::string, std::string>> t = {
      {"web_scraper",
       {"Fetch a URL and extract its title and visible text",
        "import re, urllib.request\n\n"
        "def main(input_data):\n"
        "    url = input_data.get('url') or CONFIG.get('url', '')\n"
        "    html = urllib.request.urlopen(url, timeout=20).read().decode('utf-8', 'replace')\n"
        "    title = re.search(r'<title>(.*?)</title>', html, re.S | re.I)\n"
        "    text = re.sub(r'<[^>]+>', ' ', html)\n"
        "    text = re.sub(r'\\s+', ' ', text).strip()\n"
        "    n = int(input_data.get('max_length', CONFIG.get('max_length', 2000)))\n"
        "    return {'url': url, 'title': title.group(1).strip() if title else '', 'text': text[:n]}\n"}},
      {"log_analyzer",
       {"Count error / warning lines and top messages in a log file",
        "import collections\n\n"
        "def main(input_data):\n"
        "    path = input_data.get('path') or CONFIG.get('path', '/var/log/syslog')\n"
        "    pats = CONFIG.get('patterns', ['ERROR', 'WARN', 'CRITICAL'])\n"
        "    counts = collections.Counter(); top = collections.Counter()\n"
        "    with open(path, errors='replace') as f:\n"
        "        for line in f:\n"
        "            for p in pats:\n"
        "                if p in line:\n"
        "                    counts[p] += 1; top[line.strip()[-120:]] += 1\n"
        "    return {'path': path, 'counts': dict(counts), 'top': top.most_common(10)}\n"}},
      {"file_processor",
       {"Line / word / byte statistics of text files matching a pattern",
        "import glob, os\n\n"
        "def main(input_data):\n"
        "    pattern = input_data.get('pattern') or CONFIG.get('pattern', '/tmp/*.txt')\n"
        "    out = []\n"
        "    for p in sorted(glob.glob(pattern))[:200]:\n"
        "        with open(p, errors='replace') as f:\n"
        "            data = f.read()\n"
        "        out.append({'path': p, 'lines': data.count('\\n'), 'words': len(data.split()), 'bytes': os.path.getsize(p)})\n"
        "    return {'files': out, 'count': len(out)}\n"}},
      {"api_client",
       {"Call a JSON HTTP API",
        "import json, urllib.request\n\n"
        "def main(input_data):\n"
        "    url = input_data.get('url') or CONFIG.get('base_url', '')\n"
        "    method = input_data.get('method', CONFIG.get('method', 'GET'))\n"
        "    body = input_data.get('body')\n"
        "    req = urllib.request.Request(url, method=method, data=json.dumps(body).encode() if body is not None else None,\n"
        "                                 headers={'Content-Type': 'application/json', **CONFIG.get('headers', {})})\n"
        "    with urllib.request.urlopen(req, timeout=20) as r:\n"
        "        raw = r.read().decode('utf-8', 'replace')\n"
        "        try:\n"
        "            return {'status': r.status, 'data': json.loads(raw)}\n"
        "        except ValueError:\n"
        "            return {'status': r.status, 'raw': raw[:4000]}\n"}},
  };
  return t;
}

std::string container_rt() {
  for (const char* r : {"podman", "docker"})
    if (have_cmd(r)) return r;
  tool_fail("no container runtime (podman / docker) available");
}
std::string valid_cname(const std::string& n) {
  static const std::regex re("^[A-Za-z0-9][A-Za-z0-9_.-]{0,127}$");
  if (!std::regex_match(n, re)) tool_fail("invalid container name: " + n);
  return n;
}

std::string scaffold_readme(const std::string& name, const std::string& desc) {
  return "# " + name + "\n\n" + (desc.empty() ? "Generated by aiOS." : desc) + "\n";
}

}  // namespace

Json plugin_validate(const std::string& code) {
  Json findings = Json::array();
  int total = 0, line_no = 0;
  for (auto& line : split(code, '\n')) {
    ++line_no;
    const std::string t = trim(line);
    if (starts_with(t, "#")) continue;
    for (auto& d : kDangerous) {
      if (t.find(d[0]) != std::string::npos) {
        findings.push(Json::object(
            {{"pattern", std::string(d[0])}, {"risk", std::atoi(d[1])}, {"description", std::string(d[2])},
             {"line_number", line_no}}));
        total += std::atoi(d[1]);
      }
    }
  }
  total = std::min(total, 100);
  const char* rec = total == 0   ? "Code appears safe"
                    : total < 30 ? "Low risk - minor concerns noted"
                    : total < 70 ? "Medium risk - review findings before deployment"
                                 : "High risk - code contains dangerous patterns and should be rejected";
  return Json::object({{"safe", total < 70}, {"risk_score", total}, {"findings", findings}, {"recommendation", rec}});
}

std::string plugin_wrapper(const std::string& user_code) {
  return "# aiOS plugin (generated wrapper: stdin JSON -> main(input_data) -> stdout JSON)\n"
         "import json as _aios_json, sys as _aios_sys\n"
         "CONFIG = {}\n\n" +
         user_code +
         "\n\nif __name__ == '__main__':\n"
         "    _raw = _aios_sys.stdin.read()\n"
         "    _data = _aios_json.loads(_raw) if _raw.strip() else {}\n"
         "    _out = main(_data)\n"
         "    print(_aios_json.dumps(_out if isinstance(_out, dict) else {'result': _out}, default=str))\n";
}

void add_dev_tools(std::vector<ToolSpec>& v) {
  // ---------------------------------------------------------------------------------- web
  add(v, "web.http_request", "HTTP request with method, headers, body and authentication", {"web.http"}, "medium", true,
      false, 30000, {"net_read", "net_write"}, [](const Json& in, ToolContext&) {
        const std::string url = http_url(in), method = lower(in.get_str("method", "GET"));
        std::string m = method;
        for (auto& c : m) c = (char)toupper(c);
        static const std::set<std::string> ok = {"GET", "POST", "PUT", "PATCH", "DELETE", "HEAD", "OPTIONS"};
        if (!ok.count(m)) tool_fail("unsupported method " + m);
        const Json& b = in["body"];
        HttpResp r = curl_req(m, url, in["headers"], b.is_null() ? "" : (b.is_str() ? b.as_str() : b.dump()),
                              in.get_str("auth_bearer"), (int)in.get_int("timeout_secs", 30), in.get_bool("follow_redirects", true));
        if (!r.err.empty()) tool_fail("request failed: " + r.err);
        return Json::object({{"status", r.status}, {"body", r.body}, {"method", m}, {"url", url}});
      });
  add(v, "web.scrape", "Fetch a page and extract its title and text (optionally only a tag's content)", {"web.read"},
      "low", true, false, 30000, {"net_read"}, [](const Json& in, ToolContext&) {
        const std::string url = http_url(in);
        HttpResp r = curl_req("GET", url, Json::object(), "", "", 25, true);
        if (!r.err.empty()) tool_fail("request failed: " + r.err);
        std::smatch m;
        std::string title;
        if (std::regex_search(r.body, m, std::regex("<title[^>]*>([\\s\\S]*?)</title>", std::regex::icase)))
          title = strip_html(m[1]);
        std::string text;
        const std::string sel = in.get_str("selector");
        static const std::regex tag_re("^[a-zA-Z][a-zA-Z0-9]*$");
        if (!sel.empty() && std::regex_match(sel, tag_re)) {
          const std::regex re("<" + sel + "[^>]*>([\\s\\S]*?)</" + sel + ">", std::regex::icase);
          for (auto it = std::sregex_iterator(r.body.begin(), r.body.end(), re); it != std::sregex_iterator(); ++it)
            text += strip_html((*it)[1]) + "\n";
        } else {
          text = strip_html(r.body);
        }
        const size_t maxl = (size_t)in.get_int("max_length", 5000);
        const bool trunc = text.size() > maxl;
        return Json::object({{"url", url},
                             {"title", title},
                             {"text", trunc ? text.substr(0, maxl) : text},
                             {"content_length", (int64_t)text.size()},
                             {"truncated", trunc}});
      });
  add(v, "web.webhook", "POST a JSON payload to a webhook (optional HMAC-SHA256 signature)", {"web.write"}, "medium",
      false, false, 15000, {"net_write"}, [](const Json& in, ToolContext&) {
        const std::string url = http_url(in);
        const Json& p = in["payload"];
        const std::string body = p.is_str() ? p.as_str() : p.dump();
        Json headers = in["headers"].is_obj() ? in["headers"] : Json::object();
        headers.set("Content-Type", "application/json");
        const std::string secret = in.get_str("secret");
        if (!secret.empty()) {
          unsigned char md[32];
          unsigned int len = 0;
          HMAC(EVP_sha256(), secret.data(), (int)secret.size(), (const unsigned char*)body.data(), body.size(), md, &len);
          std::string hex;
          static const char* hx = "0123456789abcdef";
          for (unsigned i = 0; i < len; ++i) {
            hex += hx[md[i] >> 4];
            hex += hx[md[i] & 15];
          }
          headers.set("X-Signature-256", "sha256=" + hex);
        }
        HttpResp r = curl_req("POST", url, headers, body, "", 12, true);
        return Json::object({{"success", r.ok}, {"status", r.status}, {"response_body", r.body.substr(0, 4000)},
                             {"url", url}, {"error", r.err}});
      });
  add(v, "web.download", "Download a URL to a file", {"web.http", "fs.write"}, "medium", false, true, 120000,
      {"net_read", "fs_write"}, [](const Json& in, ToolContext&) {
        const std::string url = http_url(in), dst = abs_path(in, "destination");
        if (in.get_bool("create_dirs", true)) mkdirs(dst.substr(0, dst.rfind('/')));
        const int t = (int)in.get_int("timeout_secs", 110);
        CmdResult r = sh({"curl", "-sS", "-L", "--fail", "--max-time", std::to_string(t), "-o", dst, url}, t * 1000 + 5000);
        if (r.exit_code != 0) tool_fail("download failed: " + trim(r.err));
        struct stat st;
        ::stat(dst.c_str(), &st);
        return Json::object({{"success", true}, {"url", url}, {"destination", dst}, {"size_bytes", (int64_t)st.st_size}});
      });
  add(v, "web.api_call", "Call a JSON API (query params, bearer auth); parses the JSON response", {"web.http"},
      "medium", true, false, 30000, {"net_read", "net_write"}, [](const Json& in, ToolContext&) {
        std::string url = http_url(in);
        if (in["query_params"].is_obj() && in["query_params"].size()) {
          std::string q;
          for (auto& kv : in["query_params"].as_obj()) {
            std::string val = kv.second.str_or(kv.second.dump()), enc;
            for (unsigned char c : val) {
              if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') enc += (char)c;
              else {
                char b[4];
                std::snprintf(b, sizeof b, "%%%02X", c);
                enc += b;
              }
            }
            q += (q.empty() ? "" : "&") + kv.first + "=" + enc;
          }
          url += (url.find('?') == std::string::npos ? "?" : "&") + q;
        }
        std::string m = in.get_str("method", "GET");
        for (auto& c : m) c = (char)toupper(c);
        Json headers = in["headers"].is_obj() ? in["headers"] : Json::object();
        const Json& b = in["body"];
        if (!b.is_null() && !headers.has("Content-Type")) headers.set("Content-Type", "application/json");
        HttpResp r = curl_req(m, url, headers, b.is_null() ? "" : (b.is_str() ? b.as_str() : b.dump()),
                              in.get_str("auth_bearer"), (int)in.get_int("timeout_secs", 30), true);
        if (!r.err.empty()) tool_fail("request failed: " + r.err);
        Json data;
        Json::try_parse(r.body, data);
        return Json::object({{"status", r.status}, {"success", r.ok}, {"data", data}, {"raw_body", r.body.substr(0, 8000)},
                             {"url", url}});
      });

  // ---------------------------------------------------------------------------------- git
  add(v, "git.init", "Initialise a repository", {"git.write"}, "low", false, true, 5000, {"git_write"},
      [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        mkdirs(p);
        std::vector<std::string> a{"init"};
        if (in.get_bool("bare")) a.push_back("--bare");
        git_ok(p, a);
        return Json::object({{"success", true}, {"path", p}});
      });
  add(v, "git.clone", "Clone a repository", {"git.write", "net.read"}, "medium", false, true, 120000,
      {"git_write", "net_read"}, [](const Json& in, ToolContext&) {
        const std::string url = req_str(in, "url"), dst = abs_path(in, "destination");
        if (starts_with(url, "-") || starts_with(url, "ext::")) tool_fail("invalid url");
        std::vector<std::string> a{"git", "clone"};
        if (in.has("branch")) {
          a.push_back("--branch");
          a.push_back(valid_ref(in.get_str("branch")));
        }
        if (in.get_int("depth", 0) > 0) {
          a.push_back("--depth");
          a.push_back(std::to_string(in.get_int("depth")));
        }
        a.push_back("--");
        a.push_back(url);
        a.push_back(dst);
        CmdResult r = sh(a, 115000);
        if (r.exit_code != 0) tool_fail("git clone failed: " + trim(r.err));
        return Json::object({{"success", true}, {"url", url}, {"destination", dst}});
      });
  add(v, "git.add", "Stage files", {"git.write"}, "low", true, true, 5000, {"git_write"},
      [](const Json& in, ToolContext&) {
        const std::string r = repo(in);
        std::vector<std::string> a{"add"};
        Json staged = Json::array();
        if (in.get_bool("all") || !in["files"].size()) {
          a.push_back("-A");
        } else {
          a.push_back("--");
          for (auto& f : in["files"].as_arr()) {
            a.push_back(f.as_str());
            staged.push(f);
          }
        }
        git_ok(r, a);
        if (!staged.size())
          for (auto& l : split(git(r, {"diff", "--cached", "--name-only"}).out, '\n'))
            if (!trim(l).empty()) staged.push(trim(l));
        return Json::object({{"success", true}, {"files_staged", staged}});
      });
  add(v, "git.commit", "Commit staged changes", {"git.write"}, "low", false, false, 10000, {"git_write"},
      [](const Json& in, ToolContext&) {
        const std::string r = repo(in), msg = req_str(in, "message");
        std::vector<std::string> a{"-c", "user.name=aiOS", "-c", "user.email=aios@localhost", "commit", "-m", msg};
        const std::string author = in.get_str("author");
        if (!author.empty()) a.push_back("--author=" + author);
        git_ok(r, a);
        return Json::object({{"success", true}, {"commit_hash", trim(git(r, {"rev-parse", "HEAD"}).out)}, {"message", msg}});
      });
  add(v, "git.push", "Push to a remote", {"git.write", "net.write"}, "high", false, false, 60000,
      {"git_write", "net_write"}, [](const Json& in, ToolContext&) {
        const std::string r = repo(in), remote = valid_ref(in.get_str("remote", "origin"));
        std::vector<std::string> a{"push", remote};
        if (in.has("branch")) a.push_back(valid_ref(in.get_str("branch")));
        git_ok(r, a, 55000);
        return Json::object({{"success", true}, {"remote", remote}, {"branch", in.get_str("branch")}});
      });
  add(v, "git.pull", "Pull from a remote", {"git.write", "net.read"}, "medium", false, false, 60000,
      {"git_write", "net_read"}, [](const Json& in, ToolContext&) {
        const std::string r = repo(in), remote = valid_ref(in.get_str("remote", "origin"));
        std::vector<std::string> a{"pull", "--ff-only", remote};
        if (in.has("branch")) a.push_back(valid_ref(in.get_str("branch")));
        CmdResult c = git_ok(r, a, 55000);
        return Json::object({{"success", true}, {"remote", remote}, {"output", trim(c.out)}});
      });
  add(v, "git.branch", "List, create, switch or delete branches", {"git.write"}, "low", true, true, 5000,
      {"git_write"}, [](const Json& in, ToolContext&) {
        const std::string r = repo(in), action = in.get_str("action", "list");
        if (action == "create") git_ok(r, {"branch", valid_ref(req_str(in, "name"))});
        else if (action == "switch" || action == "checkout") git_ok(r, {"checkout", valid_ref(req_str(in, "name"))});
        else if (action == "delete") git_ok(r, {"branch", "-d", valid_ref(req_str(in, "name"))});
        else if (action != "list") tool_fail("unknown action: " + action);
        Json br = Json::array();
        for (auto& l : split(git(r, {"branch", "--format=%(refname:short)"}).out, '\n'))
          if (!trim(l).empty()) br.push(trim(l));
        return Json::object({{"success", true}, {"action", action}, {"branches", br},
                             {"current", trim(git(r, {"rev-parse", "--abbrev-ref", "HEAD"}).out)}});
      });
  add(v, "git.status", "Working tree status", {"git.read"}, "low", true, false, 5000, {"git_read"},
      [](const Json& in, ToolContext&) {
        const std::string r = repo(in);
        CmdResult c = git_ok(r, {"status", "--porcelain=v1", "--branch"});
        Json staged = Json::array(), modified = Json::array(), untracked = Json::array();
        std::string branch;
        for (auto& l : split(c.out, '\n')) {
          if (l.size() < 3) continue;
          if (starts_with(l, "## ")) {
            branch = l.substr(3, l.find("...") == std::string::npos ? std::string::npos : l.find("...") - 3);
            continue;
          }
          const std::string f = l.substr(3);
          if (l[0] == '?') untracked.push(f);
          else {
            if (l[0] != ' ') staged.push(f);
            if (l[1] != ' ') modified.push(f);
          }
        }
        return Json::object({{"clean", staged.size() + modified.size() + untracked.size() == 0}, {"branch", branch},
                             {"staged", staged}, {"modified", modified}, {"untracked", untracked}});
      });
  add(v, "git.log", "Recent commits", {"git.read"}, "low", true, false, 5000, {"git_read"},
      [](const Json& in, ToolContext&) {
        const std::string r = repo(in);
        const int n = (int)std::max<int64_t>(1, std::min<int64_t>(500, in.get_int("count", 10)));
        CmdResult c = git_ok(r, {"log", "-n", std::to_string(n), "--pretty=format:%H%x1f%an%x1f%aI%x1f%s"});
        Json e = Json::array();
        for (auto& l : split(c.out, '\n')) {
          auto f = split(l, '\x1f');
          if (f.size() == 4) e.push(Json::object({{"hash", f[0]}, {"author", f[1]}, {"date", f[2]}, {"message", f[3]}}));
        }
        return Json::object({{"entries", e}});
      });
  add(v, "git.diff", "Diff of the working tree, the staging area or a commit", {"git.read"}, "low", true, false, 10000,
      {"git_read"}, [](const Json& in, ToolContext&) {
        const std::string r = repo(in);
        std::vector<std::string> a{"diff"}, names{"diff", "--name-only"};
        if (in.get_bool("staged")) {
          a.push_back("--cached");
          names.push_back("--cached");
        }
        if (in.has("commit")) {
          a.push_back(valid_ref(in.get_str("commit")));
          names.push_back(valid_ref(in.get_str("commit")));
        }
        CmdResult c = git_ok(r, a);
        Json files = Json::array();
        for (auto& l : split(git(r, names).out, '\n'))
          if (!trim(l).empty()) files.push(trim(l));
        return Json::object({{"diff", c.out.substr(0, 200000)}, {"files_changed", files}});
      });

  // ---------------------------------------------------------------------------------- code
  add(v, "code.scaffold", "Create a project skeleton (python, node, rust, cpp, hip) with README", {"fs.write", "code.gen"},
      "medium", false, true, 15000, {"fs_write", "code_gen"}, [](const Json& in, ToolContext&) {
        const std::string name = req_str(in, "name"), type = lower(in.get_str("project_type", "python"));
        static const std::regex nre("^[A-Za-z][A-Za-z0-9_-]{0,63}$");
        if (!std::regex_match(name, nre)) tool_fail("invalid project name");
        const std::string base = in.has("path") ? abs_path(in, "path") : std::string("/tmp");
        const std::string root = base + "/" + name;
        const std::string desc = in.get_str("description");
        std::map<std::string, std::string> files{{"README.md", scaffold_readme(name, desc)}, {".gitignore", "build/\n__pycache__/\n"}};
        std::string mod = name;
        std::replace(mod.begin(), mod.end(), '-', '_');
        if (type == "python") {
          files["pyproject.toml"] = "[project]\nname = \"" + name + "\"\nversion = \"0.1.0\"\n";
          files[mod + "/__init__.py"] = "\"\"\"" + (desc.empty() ? name : desc) + "\"\"\"\n";
          files[mod + "/main.py"] = "def main():\n    print(\"hello from " + name + "\")\n\n\nif __name__ == \"__main__\":\n    main()\n";
          files["tests/test_main.py"] = "from " + mod + ".main import main\n\n\ndef test_main():\n    main()\n";
        } else if (type == "node") {
          files["package.json"] = "{\n  \"name\": \"" + name + "\",\n  \"version\": \"0.1.0\",\n  \"main\": \"index.js\"\n}\n";
          files["index.js"] = "console.log('hello from " + name + "');\n";
        } else if (type == "rust") {
          files["Cargo.toml"] = "[package]\nname = \"" + mod + "\"\nversion = \"0.1.0\"\nedition = \"2021\"\n";
          files["src/main.rs"] = "fn main() {\n    println!(\"hello from " + name + "\");\n}\n";
        } else if (type == "cpp" || type == "hip") {
          const bool hip = type == "hip";
          files["CMakeLists.txt"] = "cmake_minimum_required(VERSION 3.21)\nproject(" + mod + (hip ? " LANGUAGES CXX HIP)\n" : " CXX)\n") +
                                    "add_executable(" + mod + (hip ? " src/main.hip)\n" : " src/main.cpp)\n");
          files[hip ? "src/main.hip" : "src/main.cpp"] =
              hip ? "#include <hip/hip_runtime.h>\n#include <cstdio>\n__global__ void k(float* y) { y[threadIdx.x] = threadIdx.x; }\n"
                    "int main() {\n  float* y;\n  hipMalloc(&y, 64 * sizeof(float));\n  k<<<1, 64>>>(y);\n  hipDeviceSynchronize();\n"
                    "  std::printf(\"ok\\n\");\n  return 0;\n}\n"
                  : "#include <cstdio>\nint main() {\n  std::printf(\"hello from " + name + "\\n\");\n  return 0;\n}\n";
        } else {
          tool_fail("unsupported project_type: " + type);
        }
        Json created = Json::array();
        for (auto& kv : files) {
          const std::string p = root + "/" + kv.first;
          mkdirs(p.substr(0, p.rfind('/')));
          std::ofstream f(p);
          f << kv.second;
          created.push(p);
        }
        return Json::object({{"success", true}, {"path", root}, {"files_created", created}, {"project_type", type}});
      });
  add(v, "code.generate", "Write a source-file skeleton for a described component", {"code.gen"}, "medium", false, true,
      30000, {"code_gen"}, [](const Json& in, ToolContext&) {
        const std::string fp = abs_path(in, "file_path"), desc = in.get_str("description");
        std::string lang = lower(in.get_str("language"));
        if (lang.empty()) {
          const std::string ext = fp.substr(fp.rfind('.') + 1);
          lang = ext == "py" ? "python" : ext == "rs" ? "rust" : ext == "js" ? "javascript" : ext == "sh" ? "bash"
               : (ext == "cpp" || ext == "cc" || ext == "h") ? "cpp" : ext == "hip" ? "hip" : "text";
        }
        std::string body;
        if (in.has("content")) body = in.get_str("content");
        else if (lang == "python") body = "\"\"\"" + desc + "\"\"\"\n\n\ndef main():\n    raise NotImplementedError\n";
        else if (lang == "bash") body = "#!/usr/bin/env bash\n# " + desc + "\nset -euo pipefail\n";
        else if (lang == "rust") body = "//! " + desc + "\n\nfn main() {}\n";
        else if (lang == "javascript") body = "// " + desc + "\n'use strict';\n";
        else if (lang == "cpp" || lang == "hip") body = "// " + desc + "\n#include <cstdio>\n";
        else body = desc + "\n";
        if (in.get_bool("create_dirs", true)) mkdirs(fp.substr(0, fp.rfind('/')));
        std::ofstream f(fp);
        if (!f) tool_fail("cannot write " + fp);
        f << body;
        return Json::object({{"success", true}, {"file_path", fp}, {"language", lang},
                             {"lines", (int64_t)std::count(body.begin(), body.end(), '\n')},
                             {"generated_by", in.has("content") ? "caller" : "template"}});
      });

  // ---------------------------------------------------------------------------------- self
  add(v, "self.inspect", "Framework version, components, git revision and configuration", {"self.read"}, "low", true,
      false, 10000, {"self_read"}, [](const Json& in, ToolContext& ctx) {
        const std::string src = in.get_str("source_path", ctx.paths->source_dir);
        Json comps = Json::array();
        for (const char* c : {"aios-runtime (MI355X HIP engine)", "aios-tools", "aios-memory", "aios-orchestrator",
                              "aios-api-gateway", "aios-init"})
          comps.push(c);
        std::string rev, branch;
        if (!src.empty() && have_cmd("git")) {
          rev = trim(git(src, {"rev-parse", "HEAD"}).out);
          branch = trim(git(src, {"rev-parse", "--abbrev-ref", "HEAD"}).out);
        }
        return Json::object({{"version", "0.1.0"}, {"components", comps}, {"git_revision", rev}, {"git_branch", branch},
                             {"source_path", src}, {"tools", (int64_t)ctx.svc->tool_count()},
                             {"data_dir", ctx.paths->data_dir}});
      });
  add(v, "self.health", "Service reachability, disk usage and uptime", {"self.read"}, "low", true, false, 15000,
      {"self_read"}, [](const Json& in, ToolContext&) {
        Json services = Json::array(), issues = Json::array();
        bool healthy = true;
        if (in.get_bool("check_services", true)) {
          static const std::pair<const char*, int> svcs[] = {{"orchestrator", 50051}, {"tools", 50052}, {"memory", 50053},
                                                             {"api-gateway", 50054}, {"runtime", 50055}};
          for (auto& s : svcs) {
            ToolContext* unused = nullptr;
            (void)unused;
            CmdLimits l;
            // TCP probe (health.rs semantics): connect to 127.0.0.1:<port>
            int fd = ::socket(AF_INET, SOCK_STREAM, 0);
            sockaddr_in sa{};
            sa.sin_family = AF_INET;
            sa.sin_port = htons((uint16_t)s.second);
            sa.sin_addr.s_addr = htonl(0x7f000001);
            const bool up = fd >= 0 && ::connect(fd, (sockaddr*)&sa, sizeof sa) == 0;
            if (fd >= 0) ::close(fd);
            services.push(Json::object({{"name", std::string(s.first)}, {"port", s.second}, {"reachable", up}}));
            if (!up) issues.push(std::string(s.first) + " unreachable on :" + std::to_string(s.second));
          }
        }
        double pct = 0;
        bool disk_ok = true;
        if (in.get_bool("check_disk", true)) {
          struct statvfs s;
          if (::statvfs("/", &s) == 0 && s.f_blocks) {
            pct = 100.0 * (double)(s.f_blocks - s.f_bfree) / (double)s.f_blocks;
            disk_ok = pct < 90.0;
            if (!disk_ok) issues.push("disk usage above 90%");
          }
        }
        healthy = issues.size() == 0;
        double up = 0;
        try {
          up = std::stod(read_file("/proc/uptime"));
        } catch (...) {
        }
        return Json::object({{"healthy", healthy}, {"services", services}, {"disk_ok", disk_ok},
                             {"disk_usage_percent", pct}, {"uptime_seconds", (int64_t)up}, {"issues", issues}});
      });
  add(v, "self.update", "Fast-forward the framework source tree from its remote", {"self.update"}, "critical", false,
      false, 120000, {"self_update"}, [](const Json& in, ToolContext& ctx) {
        const std::string src = in.get_str("source_path", ctx.paths->source_dir);
        if (src.empty()) tool_fail("no source_path (set AIOS_SOURCE_DIR)");
        const std::string prev = trim(git_ok(src, {"rev-parse", "HEAD"}).out);
        const std::string remote = valid_ref(in.get_str("remote", "origin"));
        std::vector<std::string> a{"pull", "--ff-only", remote};
        if (in.has("branch")) a.push_back(valid_ref(in.get_str("branch")));
        CmdResult c = git(src, a, 110000);
        const std::string cur = trim(git(src, {"rev-parse", "HEAD"}).out);
        Json files = Json::array();
        if (prev != cur)
          for (auto& l : split(git(src, {"diff", "--name-only", prev, cur}).out, '\n'))
            if (!trim(l).empty()) files.push(trim(l));
        return Json::object({{"success", c.exit_code == 0}, {"previous_rev", prev}, {"current_rev", cur},
                             {"files_changed", files}, {"output", trim(c.out + c.err)}});
      });
  add(v, "self.rebuild", "Rebuild the native components (gfx950 HIP engine + control-plane core)", {"self.update"},
      "critical", false, false, 300000, {"self_update"}, [](const Json& in, ToolContext& ctx) {
        const std::string src = in.get_str("source_path", ctx.paths->source_dir);
        if (src.empty()) tool_fail("no source_path (set AIOS_SOURCE_DIR)");
        const int64_t t0 = now_ms();
        CmdResult c = sh({"python3", "-c", "import __graft_entry__ as g; g.build()"}, 290000, src);
        Json comps = Json::array();
        comps.push("aios_amd._engine");
        comps.push("aios_amd._core");
        return Json::object({{"success", c.exit_code == 0}, {"components_built", c.exit_code == 0 ? comps : Json::array()},
                             {"duration_secs", (double)(now_ms() - t0) / 1000.0},
                             {"output", (c.out + c.err).substr(0, 8000)}});
      });

  // ---------------------------------------------------------------------------------- plugin
  add(v, "plugin.create", "Create a plugin tool from Python code defining main(input_data) -> dict",
      {"plugin_manage", "fs_write"}, "high", false, true, 30000, {"plugin_manage", "fs_write"},
      [](const Json& in, ToolContext& ctx) {
        const std::string name = valid_plugin_name(req_str(in, "name"));
        Json paths = write_plugin(ctx, name, in.get_str("description"), req_str(in, "code"), in["capabilities"],
                                  in["dependencies"], in["next_plugins"], in.get_str("output_mode", "pipe"));
        Json deps_installed = Json::array();
        if (in["dependencies"].size()) deps_installed = pip_install(in["dependencies"])["installed"];
        return Json::object({{"success", true}, {"tool_name", "plugin." + name}, {"script_path", paths["script_path"]},
                             {"metadata_path", paths["metadata_path"]}, {"dependencies_installed", deps_installed}});
      });
  add(v, "plugin.list", "List plugin tools", {"plugin_read"}, "low", true, false, 5000, {"plugin_read"},
      [](const Json&, ToolContext& ctx) {
        Json pl = Json::array();
        if (DIR* d = ::opendir(ctx.paths->plugin_dir().c_str())) {
          while (dirent* e = ::readdir(d)) {
            const std::string f = e->d_name;
            if (!ends_with(f, ".meta.json")) continue;
            Json m;
            if (!Json::try_parse(read_file(ctx.paths->plugin_dir() + "/" + f), m)) continue;
            const std::string n = f.substr(0, f.size() - 10);
            pl.push(Json::object({{"tool_name", m.get_str("tool_name", "plugin." + n)},
                                  {"description", m.get_str("description")},
                                  {"script_path", ctx.paths->plugin_dir() + "/" + n + ".py"},
                                  {"dependencies", m["dependencies"]},
                                  {"created_at", m.get_str("created_at")}}));
          }
          ::closedir(d);
        }
        return Json::object({{"plugins", pl}, {"count", (int64_t)pl.size()}});
      });
  add(v, "plugin.delete", "Delete a plugin tool", {"plugin_manage"}, "high", false, false, 5000, {"plugin_manage"},
      [](const Json& in, ToolContext& ctx) {
        const std::string name = valid_plugin_name(req_str(in, "name"));
        Json deleted = Json::array();
        for (const char* ext : {".py", ".meta.json"}) {
          const std::string f = ctx.paths->plugin_dir() + "/" + name + ext;
          if (::unlink(f.c_str()) == 0) deleted.push(f);
        }
        if (!deleted.size()) tool_fail("no such plugin: " + name);
        ctx.svc->deregister_tool("plugin." + name);
        return Json::object({{"success", true}, {"deleted_files", deleted}});
      });
  add(v, "plugin.install_deps", "pip-install a plugin's Python dependencies (user site)", {"plugin_manage", "pkg_manage"},
      "high", false, false, 60000, {"plugin_manage", "pkg_manage"}, [](const Json& in, ToolContext&) {
        valid_plugin_name(req_str(in, "name"));
        Json r = pip_install(in["packages"]);
        return Json::object({{"success", r.get_str("error").empty()}, {"packages_installed", r["installed"]},
                             {"error", r.get_str("error")}});
      });
  add(v, "plugin.from_template", "Create a plugin from a template (web_scraper, log_analyzer, file_processor, api_client)",
      {"plugin_manage", "fs_write"}, "medium", false, true, 30000, {"plugin_manage", "fs_write"},
      [](const Json& in, ToolContext& ctx) {
        const std::string t = req_str(in, "template");
        auto it = templates().find(t);
        if (it == templates().end()) tool_fail("unknown template: " + t);
        const Json& cfg = in["config"];
        const std::string name = valid_plugin_name(cfg.get_str("name", in.get_str("name", t)));
        const std::string code = "CONFIG.update(" + (cfg.is_obj() ? cfg.dump() : std::string("{}")) + ")\n" +
                                 it->second.second;
        write_plugin(ctx, name, cfg.get_str("description", it->second.first), code, Json::array(), Json::array(),
                     Json::array(), "pipe");
        ctx.svc->scan_plugins();
        return Json::object({{"success", true}, {"plugin_name", name}, {"tool_name", "plugin." + name}});
      });

  // ---------------------------------------------------------------------------------- container
  add(v, "container.create", "Create and start a container", {"container.manage"}, "medium", false, true, 30000,
      {"container_manage"}, [](const Json& in, ToolContext&) {
        const std::string rt = container_rt(), image = req_str(in, "image");
        std::vector<std::string> a{rt, "run", "-d"};
        std::string name = in.get_str("name");
        if (!name.empty()) {
          a.push_back("--name");
          a.push_back(valid_cname(name));
        }
        for (auto& p : in["ports"].as_arr()) {
          a.push_back("-p");
          a.push_back(p.str_or(p.dump()));
        }
        for (auto& kv : in["env"].as_obj()) {
          a.push_back("-e");
          a.push_back(kv.first + "=" + kv.second.str_or(kv.second.dump()));
        }
        for (auto& vol : in["volumes"].as_arr()) {
          a.push_back("-v");
          a.push_back(vol.as_str());
        }
        a.push_back(image);
        CmdResult r = sh(a, 28000);
        if (r.exit_code != 0) tool_fail(rt + " run failed: " + trim(r.err));
        return Json::object({{"success", true}, {"container_id", trim(r.out)}, {"name", name}});
      });
  add(v, "container.start", "Start a container", {"container.manage"}, "low", true, true, 10000, {"container_manage"},
      [](const Json& in, ToolContext&) {
        const std::string n = valid_cname(req_str(in, "name"));
        CmdResult r = sh({container_rt(), "start", n}, 9000);
        if (r.exit_code != 0) tool_fail("start failed: " + trim(r.err));
        return Json::object({{"success", true}, {"name", n}});
      });
  add(v, "container.stop", "Stop a container", {"container.manage"}, "low", true, true, 15000, {"container_manage"},
      [](const Json& in, ToolContext&) {
        const std::string n = valid_cname(req_str(in, "name"));
        CmdResult r = sh({container_rt(), "stop", "-t", std::to_string(in.get_int("timeout", 10)), n}, 14000);
        if (r.exit_code != 0) tool_fail("stop failed: " + trim(r.err));
        return Json::object({{"success", true}, {"name", n}});
      });
  add(v, "container.list", "List containers", {"container.read"}, "low", true, false, 5000, {"container_read"},
      [](const Json& in, ToolContext&) {
        std::vector<std::string> a{container_rt(), "ps", "--format", "{{.ID}}\t{{.Names}}\t{{.Image}}\t{{.Status}}"};
        if (in.get_bool("all")) a.push_back("-a");
        CmdResult r = sh(a, 5000);
        Json cs = Json::array();
        for (auto& l : split(r.out, '\n')) {
          auto f = split(l, '\t');
          if (f.size() == 4) cs.push(Json::object({{"id", f[0]}, {"name", f[1]}, {"image", f[2]}, {"status", f[3]}}));
        }
        return Json::object({{"containers", cs}, {"total", (int64_t)cs.size()}});
      });
  add(v, "container.exec", "Run a command inside a container", {"container.manage"}, "high", false, false, 30000,
      {"container_manage"}, [](const Json& in, ToolContext&) {
        const std::string n = valid_cname(req_str(in, "name"));
        std::vector<std::string> a{container_rt(), "exec", n};
        const Json& c = in["command"];
        if (c.is_arr()) for (auto& x : c.as_arr()) a.push_back(x.as_str());
        else for (auto& w : split_ws(req_str(in, "command"))) a.push_back(w);
        CmdResult r = sh(a, 28000);
        return Json::object({{"success", r.exit_code == 0}, {"exit_code", r.exit_code}, {"stdout", r.out}, {"stderr", r.err}});
      });
  add(v, "container.logs", "Container log tail", {"container.read"}, "low", true, false, 10000, {"container_read"},
      [](const Json& in, ToolContext&) {
        const std::string n = valid_cname(req_str(in, "name"));
        CmdResult r = sh({container_rt(), "logs", "--tail", std::to_string(in.get_int("tail", 100)), n}, 9000);
        if (r.exit_code != 0) tool_fail("logs failed: " + trim(r.err));
        Json lines = Json::array();
        for (auto& l : split(r.out + r.err, '\n'))
          if (!l.empty()) lines.push(l);
        return Json::object({{"success", true}, {"name", n}, {"lines", lines}, {"total_lines", (int64_t)lines.size()}});
      });

  // ---------------------------------------------------------------------------------- email
  add(v, "email.send", "Send an email over SMTP (AIOS_SMTP_URL, AIOS_SMTP_USER, AIOS_SMTP_PASSWORD, AIOS_SMTP_FROM)",
      {"email_send"}, "medium", false, false, 30000, {"email_send"}, [](const Json& in, ToolContext&) {
        const std::string to = req_str(in, "to"), subject = in.get_str("subject"), body = in.get_str("body");
        static const std::regex mail("^[^@\\s<>]+@[^@\\s<>]+$");
        if (!std::regex_match(to, mail)) tool_fail("invalid recipient: " + to);
        const std::string from = in.get_str("from", env_or("AIOS_SMTP_FROM", "aios@localhost"));
        const std::string url = env_or("AIOS_SMTP_URL", "");
        if (url.empty()) tool_fail("SMTP not configured (set AIOS_SMTP_URL, e.g. smtps://smtp.example.com:465)");
        std::string msg = "From: " + from + "\r\nTo: " + to + "\r\n";
        if (in.has("cc")) msg += "Cc: " + in.get_str("cc") + "\r\n";
        if (in.has("reply_to")) msg += "Reply-To: " + in.get_str("reply_to") + "\r\n";
        msg += "Subject: " + subject + "\r\nContent-Type: text/plain; charset=utf-8\r\n\r\n" + body + "\r\n";
        std::vector<std::string> a{"curl", "-sS", "--url", url, "--mail-from", from, "--mail-rcpt", to, "--upload-file", "-"};
        if (in.has("cc") && std::regex_match(in.get_str("cc"), mail)) {
          a.push_back("--mail-rcpt");
          a.push_back(in.get_str("cc"));
        }
        const std::string user = env_or("AIOS_SMTP_USER", "");
        if (!user.empty()) {
          a.push_back("--user");
          a.push_back(user + ":" + env_or("AIOS_SMTP_PASSWORD", ""));
        }
        CmdResult r = sh(a, 25000, "", msg);
        if (r.exit_code != 0) tool_fail("SMTP send failed: " + trim(r.err));
        return Json::object({{"success", true}, {"message", "sent"}, {"from", from}, {"to", to}});
      });
}

}  // namespace aiosn
