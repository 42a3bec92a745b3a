// aios-init: boot + service supervisor for an aiOS MI355X node.
//
// Reference: `initd/src/{main,service,config,hardware}.rs`.  Phases:
//   1  mount /proc /sys /dev /tmp /run /dev/pts /dev/shm            (only when running as PID 1)
//   2  load config ($AIOS_CONFIG or /etc/aios/config.toml; defaults when missing)
//   3  hostname + hardware detection (CPU, RAM, AMD GPUs from /sys/class/drm + /dev/kfd) written
//      to <data_dir>/hardware.json
//   3.5 first boot (<data_dir>/.first-boot): run first_boot_script if present, else create the
//      directory layout inline
//   4  start the service DAG in topological order (orchestrator after runtime, memory, tools and
//      api-gateway), waiting for each service's TCP port (runtime 30 s -- model load -- others 10 s)
//   then supervise: reap zombies every 100 ms, check services every 10 s, restart a dead service
//   unless it failed max_restarts times within restart_window_s; SIGTERM/SIGINT stop everything
//   (SIGTERM, then SIGKILL after 10 s) and write the clean-shutdown flag.
// The services are the framework's Python daemons by default (python3 -m aios_amd.<svc>...);
// any [services.<name>] table in the config overrides command / port / deps / env.
//
// Testing hooks: --check-config prints the resolved config as JSON; --run-for S supervises for S
// seconds and exits; --no-mount / --dry-run.
#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/mount.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/utsname.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../json.h"

using aiosn::Json;

namespace {

std::atomic<bool> g_stop{false};
FILE* g_log = stderr;

void logf(const char* lvl, const std::string& msg) {
  char ts[32];
  time_t t = time(nullptr);
  strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", gmtime(&t));
  fprintf(g_log, "%s %s aios-init: %s\n", ts, lvl, msg.c_str());
  fflush(g_log);
}
#define INFO(m) logf("INFO", m)
#define WARN(m) logf("WARN", m)

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// ------------------------------------------------------------------------------ TOML subset
// tables [a.b], key = "str" | 'str' | int | float | bool | [array of scalars], # comments.
// Produces a nested Json object.
Json toml_value(const std::string& v) {
  const std::string s = trim(v);
  if (s.empty()) return Json();
  if (s[0] == '"' || s[0] == '\'') {
    const char q = s[0];
    std::string out;
    for (size_t i = 1; i < s.size() && s[i] != q; ++i) {
      if (q == '"' && s[i] == '\\' && i + 1 < s.size()) {
        ++i;
        out += s[i] == 'n' ? '\n' : s[i] == 't' ? '\t' : s[i];
      } else {
        out += s[i];
      }
    }
    return Json(out);
  }
  if (s[0] == '[') {
    Json a = Json::array();
    std::string cur;
    int depth = 0;
    char q = 0;
    for (size_t i = 1; i < s.size(); ++i) {
      char c = s[i];
      if (q) {
        cur += c;
        if (c == q) q = 0;
        continue;
      }
      if (c == '"' || c == '\'') { q = c; cur += c; continue; }
      if (c == '[') ++depth;
      if (c == ']' && depth-- == 0) break;
      if (c == ',' && depth == 0) {
        if (!trim(cur).empty()) a.push(toml_value(cur));
        cur.clear();
        continue;
      }
      cur += c;
    }
    if (!trim(cur).empty()) a.push(toml_value(cur));
    return a;
  }
  if (s == "true") return Json(true);
  if (s == "false") return Json(false);
  std::string num;
  for (char c : s)
    if (c != '_') num += c;
  char* end = nullptr;
  if (num.find_first_of(".eE") == std::string::npos) {
    long long x = strtoll(num.c_str(), &end, 10);
    if (end && *end == 0) return Json((int64_t)x);
  }
  double d = strtod(num.c_str(), &end);
  if (end && *end == 0) return Json(d);
  return Json(s);
}

std::string strip_comment(const std::string& line) {
  char q = 0;
  for (size_t i = 0; i < line.size(); ++i) {
    char c = line[i];
    if (q) { if (c == q) q = 0; continue; }
    if (c == '"' || c == '\'') q = c;
    else if (c == '#') return line.substr(0, i);
  }
  return line;
}

Json& table_at(Json& root, const std::vector<std::string>& path) {
  Json* cur = &root;
  for (auto& k : path) {
    if (!cur->has(k) || !(*cur)[k].is_obj()) cur->set(k, Json::object());
    cur = const_cast<Json*>(&(*cur)[k]);
  }
  return *cur;
}

Json parse_toml(const std::string& text) {
  Json root = Json::object();
  std::vector<std::string> table;
  std::istringstream in(text);
  std::string line, pending;
  while (std::getline(in, line)) {
    line = trim(strip_comment(line));
    if (line.empty()) continue;
    if (!pending.empty()) {  // multi-line array continuation
      pending += " " + line;
      if (std::count(pending.begin(), pending.end(), '[') > std::count(pending.begin(), pending.end(), ']')) continue;
      line = pending;
      pending.clear();
    }
    if (line[0] == '[' && line.find('=') == std::string::npos) {
      std::string name = trim(line.substr(1, line.find(']') - 1));
      table.clear();
      std::stringstream ss(name);
      std::string part;
      while (std::getline(ss, part, '.')) table.push_back(trim(part));
      table_at(root, table);
      continue;
    }
    auto eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::string key = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
    if (!key.empty() && key.front() == '"') key = key.substr(1, key.size() - 2);
    if (!val.empty() && val[0] == '[' &&
        std::count(val.begin(), val.end(), '[') > std::count(val.begin(), val.end(), ']')) {
      pending = line;
      continue;
    }
    table_at(root, table).set(key, toml_value(val));
  }
  return root;
}

// merge `over` into `base` recursively
void merge(Json& base, const Json& over) {
  for (auto& kv : over.as_obj()) {
    if (kv.second.is_obj() && base.has(kv.first) && base[kv.first].is_obj()) {
      Json sub = base[kv.first];
      merge(sub, kv.second);
      base.set(kv.first, sub);
    } else {
      base.set(kv.first, kv.second);
    }
  }
}

// ------------------------------------------------------------------------------ config
Json default_config() {
  const char* py = getenv("AIOS_PYTHON") ? getenv("AIOS_PYTHON") : "python3";
  auto svc = [&](const std::string& mod, int port, Json deps, int health_timeout) {
    return Json::object({{"command", Json(Json::Arr{Json(py), Json("-m"), Json(mod)})},
                         {"port", port}, {"depends_on", deps}, {"health_timeout_s", health_timeout},
                         {"enabled", true}});
  };
  Json none = Json::array();
  Json all4 = Json(Json::Arr{Json("aios-runtime"), Json("aios-memory"), Json("aios-tools"), Json("aios-api-gateway")});
  return Json::object({
      {"system", Json::object({{"hostname", "aios"}, {"log_level", "info"},
                               {"log_dir", "/var/log/aios"}, {"autonomy_level", "full"},
                               {"data_dir", "/var/lib/aios"}})},
      {"boot", Json::object({{"init_timeout_seconds", 120}, {"debug_shell", false},
                             {"clean_shutdown_flag", "/var/lib/aios/.clean-shutdown"},
                             {"first_boot_script", "/usr/lib/aios/first-boot.sh"}})},
      {"models", Json::object({{"model_dir", "/var/lib/aios/models"}, {"devices", Json(Json::Arr{Json(0)})},
                               {"operational", Json::object({{"file", "tinyllama-1.1b-chat-v1.0.Q4_K_M.gguf"},
                                                             {"context_length", 2048}, {"always_loaded", true}})},
                               {"tactical", Json::object({{"file", "mistral-7b-instruct-v0.2.Q4_K_M.gguf"},
                                                          {"context_length", 4096}, {"always_loaded", true}})},
                               {"strategic", Json::object({{"file", "llama-3-70b.Q4_K_M.gguf"},
                                                           {"context_length", 8192}, {"tensor_parallel", 8},
                                                           {"load_on_demand", true}})}})},
      {"supervisor", Json::object({{"check_interval_s", 10}, {"max_restarts", 5}, {"restart_window_s", 300},
                                   {"stop_timeout_s", 10}})},
      {"services", Json::object({
                       {"aios-runtime", svc("aios_amd.runtime.main", 50055, none, 30)},
                       {"aios-memory", svc("aios_amd.memory.service", 50053, none, 10)},
                       {"aios-tools", svc("aios_amd.tools.service", 50052, none, 10)},
                       {"aios-api-gateway", svc("aios_amd.gateway.service", 50054, none, 10)},
                       {"aios-orchestrator", svc("aios_amd.orchestrator.main", 50051, all4, 10)},
                   })},
  });
}

Json load_config(const std::string& path, bool& from_file) {
  Json cfg = default_config();
  from_file = false;
  std::ifstream f(path);
  if (f) {
    std::stringstream ss;
    ss << f.rdbuf();
    merge(cfg, parse_toml(ss.str()));
    from_file = true;
  }
  return cfg;
}

// ------------------------------------------------------------------------------ hardware
std::string slurp(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  return trim(ss.str());
}

Json detect_hardware() {
  Json hw = Json::object();
  int cores = 0;
  std::string model;
  {
    std::ifstream f("/proc/cpuinfo");
    std::string ln;
    while (std::getline(f, ln)) {
      if (ln.rfind("processor", 0) == 0) ++cores;
      if (model.empty() && ln.rfind("model name", 0) == 0) model = trim(ln.substr(ln.find(':') + 1));
    }
  }
  hw.set("cpu_model", model);
  hw.set("cpu_cores", cores);
  {
    std::ifstream f("/proc/meminfo");
    std::string k;
    int64_t v = 0;
    std::string unit;
    while (f >> k >> v >> unit)
      if (k == "MemTotal:") { hw.set("ram_mb", v / 1024); break; }
  }
  Json gpus = Json::array();
  if (DIR* d = opendir("/sys/class/drm")) {
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.rfind("card", 0) == 0 && n.find('-') == std::string::npos) names.push_back(n);
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    for (auto& n : names) {
      const std::string dev = "/sys/class/drm/" + n + "/device/";
      const std::string vendor = slurp(dev + "vendor");
      if (vendor != "0x1002") continue;
      Json g = Json::object({{"card", n}, {"vendor", "AMD"}, {"device_id", slurp(dev + "device")}});
      const std::string vt = slurp(dev + "mem_info_vram_total");
      if (!vt.empty()) g.set("vram_gb", (double)strtoull(vt.c_str(), nullptr, 10) / 1e9);
      gpus.push(g);
    }
  }
  hw.set("gpus", gpus);
  hw.set("kfd", access("/dev/kfd", F_OK) == 0);
  struct utsname u;
  if (uname(&u) == 0) hw.set("kernel", std::string(u.release));
  return hw;
}

// ------------------------------------------------------------------------------ boot phases
bool mounted(const std::string& target) {
  std::ifstream f("/proc/mounts");
  std::string dev, mnt, rest;
  while (f >> dev >> mnt && std::getline(f, rest))
    if (mnt == target) return true;
  return false;
}

void mount_filesystems() {
  struct M { const char *src, *tgt, *type; unsigned long flags; const char* data; };
  const M ms[] = {{"proc", "/proc", "proc", MS_NOSUID | MS_NODEV | MS_NOEXEC, nullptr},
                  {"sysfs", "/sys", "sysfs", MS_NOSUID | MS_NODEV | MS_NOEXEC, nullptr},
                  {"devtmpfs", "/dev", "devtmpfs", MS_NOSUID, "mode=0755"},
                  {"tmpfs", "/tmp", "tmpfs", MS_NOSUID | MS_NODEV, "mode=1777"},
                  {"tmpfs", "/run", "tmpfs", MS_NOSUID | MS_NODEV, "mode=0755"},
                  {"devpts", "/dev/pts", "devpts", MS_NOSUID | MS_NOEXEC, "gid=5,mode=620"},
                  {"tmpfs", "/dev/shm", "tmpfs", MS_NOSUID | MS_NODEV, "mode=1777"}};
  for (auto& m : ms) {
    mkdir(m.tgt, 0755);
    if (mounted(m.tgt)) continue;
    if (mount(m.src, m.tgt, m.type, m.flags, m.data) != 0)
      WARN(std::string("mount ") + m.tgt + " failed: " + strerror(errno));
    else
      INFO(std::string("mounted ") + m.tgt);
  }
}

void mkdirs(const std::string& p) {
  std::string cur;
  std::stringstream ss(p);
  std::string part;
  while (std::getline(ss, part, '/')) {
    if (part.empty()) { cur = "/"; continue; }
    cur += (cur.empty() || cur.back() == '/' ? "" : "/") + part;
    mkdir(cur.c_str(), 0755);
  }
}

void first_boot(const Json& cfg) {
  const std::string data = cfg["system"].get_str("data_dir", "/var/lib/aios");
  const std::string flag = data + "/.first-boot";
  if (access(flag.c_str(), F_OK) != 0) return;
  INFO("first boot detected");
  const std::string script = cfg["boot"].get_str("first_boot_script");
  bool ran = false;
  if (!script.empty() && access(script.c_str(), X_OK) == 0) {
    pid_t p = fork();
    if (p == 0) {
      execl(script.c_str(), script.c_str(), (char*)nullptr);
      _exit(127);
    }
    int st = 0;
    waitpid(p, &st, 0);
    ran = WIFEXITED(st) && WEXITSTATUS(st) == 0;
    INFO("first-boot script exited with " + std::to_string(WEXITSTATUS(st)));
  }
  if (!ran) {
    for (const char* sub : {"data", "memory", "ledger", "models", "plugins", "cache/backups", "certs", "workspace"})
      mkdirs(data + "/" + sub);
    mkdirs(cfg["system"].get_str("log_dir", "/var/log/aios"));
  }
  unlink(flag.c_str());
}

// ------------------------------------------------------------------------------ supervisor
struct Service {
  std::string name;
  std::vector<std::string> argv;
  std::vector<std::string> env;
  std::vector<std::string> deps;
  int port = 0;
  int health_timeout_s = 10;
  pid_t pid = -1;
  std::vector<int64_t> restarts;  // timestamps
  bool given_up = false;
};

bool port_open(int port) {
  int s = socket(AF_INET, SOCK_STREAM, 0);
  if (s < 0) return false;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  bool ok = connect(s, (sockaddr*)&a, sizeof a) == 0;
  close(s);
  return ok;
}

pid_t spawn(const Service& s, const std::string& log_dir) {
  pid_t p = fork();
  if (p != 0) return p;
  setsid();
  for (auto& e : s.env) putenv(strdup(e.c_str()));
  if (!log_dir.empty()) {
    const std::string lf = log_dir + "/" + s.name + ".log";
    int fd = open(lf.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
      dup2(fd, 1);
      dup2(fd, 2);
      close(fd);
    }
  }
  std::vector<char*> av;
  for (auto& a : s.argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  execvp(av[0], av.data());
  _exit(127);
}

bool alive(pid_t p) { return p > 0 && kill(p, 0) == 0; }

int64_t now_s() { return (int64_t)time(nullptr); }

void on_signal(int) { g_stop = true; }

void reap(std::vector<Service>& svcs) {
  int st;
  pid_t p;
  while ((p = waitpid(-1, &st, WNOHANG)) > 0) {
    for (auto& s : svcs)
      if (s.pid == p) {
        WARN(s.name + " (pid " + std::to_string(p) + ") exited with " +
             std::to_string(WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st)));
        s.pid = -1;
      }
  }
}

std::vector<Service> build_services(const Json& cfg) {
  std::vector<Service> out;
  for (auto& kv : cfg["services"].as_obj()) {
    const Json& j = kv.second;
    if (!j.get_bool("enabled", true)) continue;
    Service s;
    s.name = kv.first;
    for (auto& a : j["command"].as_arr()) s.argv.push_back(a.as_str());
    if (j["command"].is_str()) {
      std::stringstream ss(j.get_str("command"));
      std::string w;
      while (ss >> w) s.argv.push_back(w);
    }
    for (auto& d : j["depends_on"].as_arr()) s.deps.push_back(d.as_str());
    for (auto& e : j["env"].as_obj()) s.env.push_back(e.first + "=" + (e.second.is_str() ? e.second.as_str() : e.second.dump()));
    s.port = (int)j.get_int("port", 0);
    s.health_timeout_s = (int)j.get_int("health_timeout_s", 10);
    if (!s.argv.empty()) out.push_back(s);
  }
  return out;
}

// topological start order; services with unknown/unmet deps are reported and skipped
std::vector<size_t> start_order(const std::vector<Service>& svcs, std::vector<std::string>& unmet) {
  std::set<std::string> names, done;
  for (auto& s : svcs) names.insert(s.name);
  std::vector<size_t> order;
  std::vector<bool> placed(svcs.size(), false);
  for (size_t round = 0; round <= svcs.size(); ++round) {
    bool progress = false;
    for (size_t i = 0; i < svcs.size(); ++i) {
      if (placed[i]) continue;
      bool ok = true;
      for (auto& d : svcs[i].deps)
        if (!done.count(d)) ok = false;
      if (ok) {
        order.push_back(i);
        placed[i] = true;
        done.insert(svcs[i].name);
        progress = true;
      }
    }
    if (!progress) break;
  }
  for (size_t i = 0; i < svcs.size(); ++i)
    if (!placed[i]) unmet.push_back(svcs[i].name);
  return order;
}

void stop_all(std::vector<Service>& svcs, int timeout_s) {
  for (auto it = svcs.rbegin(); it != svcs.rend(); ++it)
    if (alive(it->pid)) kill(-it->pid, SIGTERM), kill(it->pid, SIGTERM);
  const int64_t deadline = now_s() + timeout_s;
  while (now_s() < deadline) {
    reap(svcs);
    bool any = false;
    for (auto& s : svcs) any |= alive(s.pid);
    if (!any) return;
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  for (auto& s : svcs)
    if (alive(s.pid)) kill(-s.pid, SIGKILL), kill(s.pid, SIGKILL);
  reap(svcs);
}

}  // namespace

int main(int argc, char** argv) {
  std::string cfg_path = getenv("AIOS_CONFIG") ? getenv("AIOS_CONFIG") : "/etc/aios/config.toml";
  bool check = false, dry = false, no_mount = false;
  double run_for = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--config" && i + 1 < argc) cfg_path = argv[++i];
    else if (a == "--check-config") check = true;
    else if (a == "--dry-run") dry = true;
    else if (a == "--no-mount") no_mount = true;
    else if (a == "--run-for" && i + 1 < argc) run_for = atof(argv[++i]);
    else if (a == "-h" || a == "--help") {
      printf("usage: aios-init [--config PATH] [--check-config] [--dry-run] [--no-mount] [--run-for SECONDS]\n");
      return 0;
    }
  }
  const bool pid1 = getpid() == 1;
  if (pid1 && !no_mount) mount_filesystems();  // phase 1
  bool from_file = false;
  Json cfg = load_config(cfg_path, from_file);  // phase 2
  if (check) {
    Json out = cfg;
    out.set("_config_file", from_file ? cfg_path : std::string("(defaults)"));
    std::vector<Service> svcs = build_services(cfg);
    std::vector<std::string> unmet;
    Json order = Json::array();
    for (size_t i : start_order(svcs, unmet)) order.push(svcs[i].name);
    out.set("_start_order", order);
    Json um = Json::array();
    for (auto& u : unmet) um.push(u);
    out.set("_unmet", um);
    out.set("_hardware", detect_hardware());
    printf("%s\n", out.dump(1).c_str());
    return 0;
  }
  const std::string data = cfg["system"].get_str("data_dir", "/var/lib/aios");
  const std::string log_dir = dry ? "" : cfg["system"].get_str("log_dir", "/var/log/aios");
  if (!dry) mkdirs(log_dir);
  INFO(std::string("config: ") + (from_file ? cfg_path : "defaults"));
  // phase 3
  const std::string host = cfg["system"].get_str("hostname", "aios");
  if (pid1) sethostname(host.c_str(), host.size());
  Json hw = detect_hardware();
  INFO("hardware: " + hw.dump());
  if (!dry) {
    mkdirs(data);
    std::ofstream(data + "/hardware.json") << hw.dump(1);
    first_boot(cfg);  // phase 3.5
  }
  // phase 4
  std::vector<Service> svcs = build_services(cfg);
  std::vector<std::string> unmet;
  auto order = start_order(svcs, unmet);
  if (!unmet.empty()) {
    std::string u;
    for (auto& s : unmet) u += s + " ";
    WARN("services with unmet dependencies not started: " + u);
  }
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  for (size_t i : order) {
    Service& s = svcs[i];
    std::string cmd;
    for (auto& a : s.argv) cmd += a + " ";
    if (dry) { INFO("would start " + s.name + ": " + cmd); continue; }
    s.pid = spawn(s, log_dir);
    INFO("started " + s.name + " (pid " + std::to_string(s.pid) + "): " + cmd);
    if (s.port > 0) {
      const int64_t dl = now_s() + s.health_timeout_s;
      while (!port_open(s.port) && now_s() < dl && alive(s.pid) && !g_stop)
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
      if (port_open(s.port)) INFO(s.name + " online on :" + std::to_string(s.port));
      else WARN(s.name + " health check failed, continuing");
    }
  }
  if (dry) return 0;
  INFO("boot complete: " + std::to_string(order.size()) + " services");
  const Json sup = cfg["supervisor"];
  const int check_s = (int)sup.get_int("check_interval_s", 10), max_restarts = (int)sup.get_int("max_restarts", 5);
  const int window = (int)sup.get_int("restart_window_s", 300), stop_timeout = (int)sup.get_int("stop_timeout_s", 10);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds((int64_t)(run_for * 1000));
  auto next_check = std::chrono::steady_clock::now() + std::chrono::seconds(check_s);
  while (!g_stop) {
    reap(svcs);
    const auto now = std::chrono::steady_clock::now();
    if (run_for > 0 && now >= t_end) break;
    if (now >= next_check) {
      next_check = now + std::chrono::seconds(check_s);
      for (auto& s : svcs) {
        if (s.given_up || alive(s.pid) || std::find(order.begin(), order.end(), (size_t)(&s - &svcs[0])) == order.end())
          continue;
        const int64_t t = now_s();
        s.restarts.erase(std::remove_if(s.restarts.begin(), s.restarts.end(),
                                        [&](int64_t x) { return t - x > window; }),
                         s.restarts.end());
        if ((int)s.restarts.size() >= max_restarts) {
          WARN(s.name + " failed " + std::to_string(max_restarts) + " times in " + std::to_string(window) +
               "s; giving up");
          s.given_up = true;
          continue;
        }
        s.restarts.push_back(t);
        s.pid = spawn(s, log_dir);
        INFO("restarted " + s.name + " (pid " + std::to_string(s.pid) + ", attempt " +
             std::to_string(s.restarts.size()) + ")");
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  INFO("shutting down");
  stop_all(svcs, stop_timeout);
  const std::string flag = cfg["boot"].get_str("clean_shutdown_flag", data + "/.clean-shutdown");
  std::ofstream(flag) << now_s() << "\n";
  INFO("clean shutdown");
  if (pid1) {
    sync();
    for (;;) pause();
  }
  return 0;
}
