// net (5), firewall (3), pkg (5), monitor (7), hw (1) and sec (10) tools.
// Reference: tools/src/{net,firewall,pkg,monitor,hw,sec}/*.rs (SURVEY §2.4 per-tool table).
#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <grp.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <pwd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <regex>
#include <set>
#include <thread>

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

CmdResult sh(const std::vector<std::string>& argv, int timeout_ms = 15000) {
  CmdLimits l;
  l.timeout_ms = timeout_ms;
  return run_cmd(argv, l);
}

std::string valid_host(const std::string& h) {
  static const std::regex re("^[A-Za-z0-9.:_-]{1,253}$");
  if (!std::regex_match(h, re)) tool_fail("invalid host: " + h);
  return h;
}
std::string valid_pkg(const std::string& p) {
  static const std::regex re("^[A-Za-z0-9][A-Za-z0-9.+_:~-]{0,127}$");
  if (!std::regex_match(p, re)) tool_fail("invalid package name: " + p);
  return p;
}

// TCP connect with timeout; returns connect latency in ms or -1
double tcp_connect_ms(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  double out = -1;
  for (addrinfo* ai = res; ai && out < 0; ai = ai->ai_next) {
    const int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) continue;
    const int64_t t0 = now_ms();
    int rc = connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      if (poll(&p, 1, timeout_ms) == 1) {
        int err = 0;
        socklen_t len = sizeof err;
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
        rc = err == 0 ? 0 : -1;
      } else {
        rc = -1;
      }
    }
    if (rc == 0) out = (double)(now_ms() - t0);
    close(fd);
  }
  freeaddrinfo(res);
  return out;
}

std::string pkg_manager() {
  for (const char* m : {"apt-get", "dnf", "pacman"})
    if (have_cmd(m)) return m;
  tool_fail("no supported package manager (apt-get, dnf, pacman)");
}

std::map<std::string, double> meminfo() {
  std::map<std::string, double> m;
  std::ifstream f("/proc/meminfo");
  std::string k;
  double v;
  std::string unit;
  while (f >> k >> v) {
    std::getline(f, unit);
    if (!k.empty() && k.back() == ':') k.pop_back();
    m[k] = v;  // kB
  }
  return m;
}

std::vector<uint64_t> cpu_times() {
  std::ifstream f("/proc/stat");
  std::string cpu;
  f >> cpu;
  std::vector<uint64_t> t;
  uint64_t x;
  for (int i = 0; i < 8 && (f >> x); ++i) t.push_back(x);
  return t;
}

double cpu_percent(int sample_ms) {
  auto a = cpu_times();
  std::this_thread::sleep_for(std::chrono::milliseconds(sample_ms));
  auto b = cpu_times();
  if (a.size() < 4 || b.size() < 4) return 0;
  uint64_t ta = 0, tb = 0;
  for (auto x : a) ta += x;
  for (auto x : b) tb += x;
  const uint64_t ia = a[3] + (a.size() > 4 ? a[4] : 0), ib = b[3] + (b.size() > 4 ? b[4] : 0);
  const double dt = (double)(tb - ta), di = (double)(ib - ia);
  return dt > 0 ? 100.0 * (dt - di) / dt : 0;
}

Json net_dev(const std::string& iface) {
  std::ifstream f("/proc/net/dev");
  std::string line;
  Json all = Json::object();
  while (std::getline(f, line)) {
    const auto c = line.find(':');
    if (c == std::string::npos) continue;
    const std::string name = trim(line.substr(0, c));
    auto v = split_ws(line.substr(c + 1));
    if (v.size() < 10) continue;
    Json o = Json::object({{"rx_bytes", (int64_t)std::stoll(v[0])},
                           {"rx_packets", (int64_t)std::stoll(v[1])},
                           {"tx_bytes", (int64_t)std::stoll(v[8])},
                           {"tx_packets", (int64_t)std::stoll(v[9])}});
    if (!iface.empty() && name == iface) return o;
    all.set(name, o);
  }
  if (!iface.empty()) tool_fail("no such interface: " + iface);
  // aggregate over non-loopback interfaces
  int64_t rb = 0, rp = 0, tb = 0, tp = 0;
  for (auto& kv : all.as_obj()) {
    if (kv.first == "lo") continue;
    rb += kv.second.get_int("rx_bytes");
    rp += kv.second.get_int("rx_packets");
    tb += kv.second.get_int("tx_bytes");
    tp += kv.second.get_int("tx_packets");
  }
  return Json::object({{"rx_bytes", rb}, {"tx_bytes", tb}, {"rx_packets", rp}, {"tx_packets", tp}, {"interfaces", all}});
}

// listening TCP ports from /proc/net/tcp{,6}
std::set<int> listening_ports() {
  std::set<int> ports;
  for (const char* f : {"/proc/net/tcp", "/proc/net/tcp6"}) {
    std::ifstream in(f);
    std::string line;
    std::getline(in, line);
    while (std::getline(in, line)) {
      auto v = split_ws(line);
      if (v.size() < 4 || v[3] != "0A") continue;  // TCP_LISTEN
      const auto c = v[1].rfind(':');
      if (c != std::string::npos) ports.insert((int)std::stoul(v[1].substr(c + 1), nullptr, 16));
    }
  }
  return ports;
}

void walk(const std::string& dir, int depth, const std::function<void(const std::string&, const struct stat&)>& fn,
          size_t& budget) {
  if (depth < 0 || budget == 0) return;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return;
  while (dirent* e = ::readdir(d)) {
    if (budget == 0) break;
    const std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    const std::string p = dir == "/" ? "/" + n : dir + "/" + n;
    struct stat st;
    if (::lstat(p.c_str(), &st) != 0) continue;
    --budget;
    fn(p, st);
    if (S_ISDIR(st.st_mode)) walk(p, depth - 1, fn, budget);
  }
  ::closedir(d);
}

std::string risk_from(int n_high, int n_med) {
  if (n_high > 0) return "high";
  if (n_med > 2) return "medium";
  return n_med > 0 ? "low" : "none";
}

// self-signed CA + server certificate through the openssl CLI (tls.rs / sec/cert_generate.rs semantics)
Json gen_certs(const std::string& service, const std::string& dir, int years) {
  if (!have_cmd("openssl")) tool_fail("openssl not available");
  mkdirs(dir);
  const std::string days = std::to_string(365 * std::max(1, years));
  const std::string ca_key = dir + "/ca.key", ca_crt = dir + "/ca.crt";
  const std::string key = dir + "/" + service + ".key", csr = dir + "/" + service + ".csr",
                    crt = dir + "/" + service + ".crt";
  auto must = [](const CmdResult& r, const char* what) {
    if (r.exit_code != 0) tool_fail(std::string(what) + " failed: " + trim(r.err));
  };
  if (!file_exists(ca_crt)) {
    must(sh({"openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout",
             ca_key, "-out", ca_crt, "-days", days, "-subj", "/CN=aiOS Root CA"}, 30000),
         "CA generation");
  }
  must(sh({"openssl", "req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout", key,
           "-out", csr, "-subj", "/CN=" + service}, 30000),
       "CSR generation");
  const std::string ext = dir + "/" + service + ".ext";
  {
    std::ofstream e(ext);
    e << "subjectAltName=DNS:localhost,DNS:" << service << ",IP:127.0.0.1\n";
  }
  must(sh({"openssl", "x509", "-req", "-in", csr, "-CA", ca_crt, "-CAkey", ca_key, "-CAcreateserial", "-out", crt,
           "-days", days, "-extfile", ext}, 30000),
       "certificate signing");
  ::chmod(key.c_str(), 0600);
  ::chmod(ca_key.c_str(), 0600);
  ::unlink(csr.c_str());
  ::unlink(ext.c_str());
  std::time_t t = std::time(nullptr);
  std::tm tm{};
  gmtime_r(&t, &tm);
  return Json::object({{"success", true},
                       {"ca_cert_path", ca_crt},
                       {"server_cert_path", crt},
                       {"server_key_path", key},
                       {"expires_year", 1900 + tm.tm_year + std::max(1, years)}});
}

Db& integrity_db(ToolContext& ctx) {
  static std::mutex mu;
  static std::map<std::string, std::unique_ptr<Db>> dbs;
  std::lock_guard<std::mutex> g(mu);
  auto& d = dbs[ctx.paths->integrity_db()];
  if (!d) {
    d = std::make_unique<Db>(ctx.paths->integrity_db());
    d->exec("CREATE TABLE IF NOT EXISTS baseline (path TEXT PRIMARY KEY, sha256 TEXT NOT NULL, size INTEGER, "
            "recorded_at INTEGER)");
  }
  return *d;
}

}  // namespace

void add_system_tools(std::vector<ToolSpec>& v) {
  // ---------------------------------------------------------------------------------- net
  add(v, "net.interfaces", "Network interfaces with IP address, MAC address and status", {"net.read"}, "low", true,
      false, 5000, {"net_read"}, [](const Json&, ToolContext&) {
        std::map<std::string, Json> ifs;
        ifaddrs* ia = nullptr;
        if (getifaddrs(&ia) == 0) {
          for (ifaddrs* p = ia; p; p = p->ifa_next) {
            const std::string name = p->ifa_name;
            Json& o = ifs[name];
            if (!o.is_obj()) o = Json::object({{"name", name}, {"ip", ""}, {"mac", ""}, {"status", "down"}});
            if (p->ifa_flags & IFF_UP) o.set("status", "up");
            if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET && o.get_str("ip").empty()) {
              char buf[INET_ADDRSTRLEN];
              inet_ntop(AF_INET, &((sockaddr_in*)p->ifa_addr)->sin_addr, buf, sizeof buf);
              o.set("ip", buf);
            }
          }
          freeifaddrs(ia);
        }
        Json arr = Json::array();
        for (auto& kv : ifs) {
          Json o = kv.second;
          try {
            o.set("mac", trim(read_file("/sys/class/net/" + kv.first + "/address", 64)));
          } catch (...) {
          }
          arr.push(o);
        }
        return Json::object({{"interfaces", arr}});
      });
  add(v, "net.ping", "Reachability and latency of a host (ICMP ping, TCP fallback)", {"net.read"}, "low", true, false,
      30000, {"net_read"}, [](const Json& in, ToolContext&) {
        const std::string host = valid_host(req_str(in, "host"));
        const int count = (int)std::max<int64_t>(1, std::min<int64_t>(10, in.get_int("count", 3)));
        if (have_cmd("ping")) {
          CmdResult r = sh({"ping", "-c", std::to_string(count), "-W", "2", host}, 5000 + count * 2500);
          std::smatch m;
          static const std::regex avg("= [0-9.]+/([0-9.]+)/");
          const bool ok = r.exit_code == 0;
          double lat = 0;
          if (std::regex_search(r.out, m, avg)) lat = std::stod(m[1]);
          return Json::object({{"success", ok}, {"latency_ms", lat}, {"method", "icmp"}});
        }
        double best = -1;
        for (int port : {443, 80, 22}) {
          best = tcp_connect_ms(host, port, 2000);
          if (best >= 0) break;
        }
        return Json::object({{"success", best >= 0}, {"latency_ms", best >= 0 ? best : 0.0}, {"method", "tcp"}});
      });
  add(v, "net.dns", "Resolve a hostname", {"net.read"}, "low", true, false, 10000, {"net_read"},
      [](const Json& in, ToolContext&) {
        const std::string h = valid_host(in.has("hostname") ? req_str(in, "hostname") : req_str(in, "host"));
        addrinfo hints{}, *res = nullptr;
        hints.ai_socktype = SOCK_STREAM;
        Json addrs = Json::array();
        std::set<std::string> seen;
        if (getaddrinfo(h.c_str(), nullptr, &hints, &res) == 0) {
          for (addrinfo* a = res; a; a = a->ai_next) {
            char buf[INET6_ADDRSTRLEN] = {0};
            if (a->ai_family == AF_INET) inet_ntop(AF_INET, &((sockaddr_in*)a->ai_addr)->sin_addr, buf, sizeof buf);
            else if (a->ai_family == AF_INET6) inet_ntop(AF_INET6, &((sockaddr_in6*)a->ai_addr)->sin6_addr, buf, sizeof buf);
            if (buf[0] && seen.insert(buf).second) addrs.push(std::string(buf));
          }
          freeaddrinfo(res);
        }
        return Json::object({{"addresses", addrs}});
      });
  add(v, "net.http_get", "HTTP GET a URL", {"net.http"}, "medium", true, false, 30000, {"net_read"},
      [](const Json& in, ToolContext&) {
        const std::string url = req_str(in, "url");
        if (!starts_with(url, "http://") && !starts_with(url, "https://")) tool_fail("url must be http(s)");
        CmdResult r = sh({"curl", "-sS", "-L", "--max-time", "25", "-w", "\n%{http_code}", url}, 30000);
        if (r.exit_code != 0) tool_fail("request failed: " + trim(r.err));
        const auto nl = r.out.rfind('\n');
        const int status = nl == std::string::npos ? 0 : std::atoi(r.out.c_str() + nl + 1);
        return Json::object({{"status", status}, {"body", r.out.substr(0, nl == std::string::npos ? 0 : nl)}});
      });
  add(v, "net.port_scan", "Check whether a TCP port is open", {"net.read"}, "medium", true, false, 10000,
      {"net_read", "net_scan"}, [](const Json& in, ToolContext&) {
        const std::string host = valid_host(req_str(in, "host"));
        const int port = (int)in.get_int("port", 0);
        if (port <= 0 || port > 65535) tool_fail("invalid port");
        return Json::object({{"open", tcp_connect_ms(host, port, (int)in.get_int("timeout_ms", 2000)) >= 0}});
      });

  // ---------------------------------------------------------------------------------- firewall (nftables)
  add(v, "firewall.rules", "List firewall rules", {"firewall.read"}, "low", true, false, 5000, {"firewall_read"},
      [](const Json&, ToolContext&) {
        Json rules = Json::array();
        if (have_cmd("nft")) {
          CmdResult r = sh({"nft", "-a", "list", "ruleset"});
          std::string chain;
          for (auto& line : split(r.out, '\n')) {
            const std::string t = trim(line);
            if (starts_with(t, "chain ")) chain = split_ws(t)[1];
            else if (!chain.empty() && contains(t, "# handle") && !starts_with(t, "type ")) {
              const auto w = split_ws(t);
              std::string action;
              for (auto& x : w)
                if (x == "accept" || x == "drop" || x == "reject") action = x;
              rules.push(Json::object({{"chain", chain}, {"rule", t}, {"action", action}}));
            }
          }
        } else if (have_cmd("iptables")) {
          CmdResult r = sh({"iptables", "-S"});
          for (auto& line : split(r.out, '\n')) {
            const auto w = split_ws(line);
            if (w.size() < 2 || w[0] != "-A") continue;
            std::string action = w.back();
            rules.push(Json::object({{"chain", w[1]}, {"rule", line}, {"action", action}}));
          }
        } else {
          tool_fail("no firewall backend (nft / iptables) available");
        }
        return Json::object({{"rules", rules}});
      });
  add(v, "firewall.add_rule", "Add an nftables rule to the aiOS table", {"firewall.manage"}, "critical", false, true,
      10000, {"firewall_read", "firewall_manage"}, [](const Json& in, ToolContext&) {
        if (!have_cmd("nft")) tool_fail("nft not available");
        const std::string chain = req_str(in, "chain"), rule = req_str(in, "rule");
        const std::string action = in.get_str("action", "accept");
        if (action != "accept" && action != "drop" && action != "reject") tool_fail("action must be accept|drop|reject");
        static const std::regex safe("^[A-Za-z0-9 ._:/,{}-]+$");
        if (!std::regex_match(rule, safe) || !std::regex_match(chain, safe)) tool_fail("rule contains unsafe characters");
        SandboxLimits lim;
        lim.timeout_ms = 10000;
        sandbox_exec("nft", {"add", "table", "inet", "aios"}, "", lim);
        sandbox_exec("nft", {"add", "chain", "inet", "aios", chain}, "", lim);
        std::vector<std::string> args{"add", "rule", "inet", "aios", chain};
        for (auto& w : split_ws(rule)) args.push_back(w);
        args.push_back(action);
        SandboxResult r = sandbox_exec("nft", args, "", lim);
        if (!r.success) tool_fail("nft failed: " + r.error);
        return Json::object({{"added", true}});
      });
  add(v, "firewall.delete_rule", "Delete the index-th rule of an aiOS chain", {"firewall.manage"}, "critical", false,
      false, 10000, {"firewall_read", "firewall_manage"}, [](const Json& in, ToolContext&) {
        if (!have_cmd("nft")) tool_fail("nft not available");
        const std::string chain = req_str(in, "chain");
        const int idx = (int)in.get_int("index", -1);
        CmdResult r = sh({"nft", "-a", "list", "chain", "inet", "aios", chain});
        std::vector<std::string> handles;
        static const std::regex hre("# handle ([0-9]+)");
        for (auto& line : split(r.out, '\n')) {
          std::smatch m;
          const std::string t = trim(line);
          if (!starts_with(t, "chain") && !starts_with(t, "type") && std::regex_search(t, m, hre)) handles.push_back(m[1]);
        }
        if (idx < 0 || idx >= (int)handles.size()) tool_fail("rule index out of range");
        SandboxLimits lim;
        SandboxResult d = sandbox_exec("nft", {"delete", "rule", "inet", "aios", chain, "handle", handles[idx]}, "", lim);
        if (!d.success) tool_fail("nft failed: " + d.error);
        return Json::object({{"deleted", true}});
      });

  // ---------------------------------------------------------------------------------- pkg
  add(v, "pkg.install", "Install a package", {"pkg.manage"}, "high", false, true, 120000, {"pkg_manage"},
      [](const Json& in, ToolContext&) {
        const std::string p = valid_pkg(req_str(in, "name")), m = pkg_manager();
        SandboxLimits lim;
        lim.timeout_ms = 115000;
        lim.cpu_seconds = 110;
        lim.mem_bytes = 2ull << 30;
        lim.allow_network = true;
        SandboxResult r = m == "apt-get" ? sandbox_exec("apt-get", {"install", "-y", p}, "", lim)
                          : m == "dnf"   ? sandbox_exec("dnf", {"install", "-y", p}, "", lim)
                                         : sandbox_exec("pacman", {"-S", "--noconfirm", p}, "", lim);
        if (!r.success) tool_fail("install failed: " + r.error);
        std::string ver;
        if (have_cmd("dpkg-query")) ver = trim(sh({"dpkg-query", "-W", "-f=${Version}", p}).out);
        return Json::object({{"installed", true}, {"version", ver}});
      });
  add(v, "pkg.remove", "Remove a package", {"pkg.manage"}, "high", false, false, 60000, {"pkg_manage"},
      [](const Json& in, ToolContext&) {
        const std::string p = valid_pkg(req_str(in, "name")), m = pkg_manager();
        SandboxLimits lim;
        lim.timeout_ms = 55000;
        lim.cpu_seconds = 50;
        lim.mem_bytes = 1ull << 30;
        SandboxResult r = m == "apt-get" ? sandbox_exec("apt-get", {"remove", "-y", p}, "", lim)
                          : m == "dnf"   ? sandbox_exec("dnf", {"remove", "-y", p}, "", lim)
                                         : sandbox_exec("pacman", {"-R", "--noconfirm", p}, "", lim);
        if (!r.success) tool_fail("remove failed: " + r.error);
        return Json::object({{"removed", true}});
      });
  add(v, "pkg.search", "Search the package index", {"pkg.read"}, "low", true, false, 30000, {"pkg_read"},
      [](const Json& in, ToolContext&) {
        const std::string q = valid_pkg(req_str(in, "query")), m = pkg_manager();
        CmdResult r = m == "apt-get" ? sh({"apt-cache", "search", q}, 25000)
                      : m == "dnf"   ? sh({"dnf", "search", "-q", q}, 25000)
                                     : sh({"pacman", "-Ss", q}, 25000);
        Json pk = Json::array();
        for (auto& line : split(r.out, '\n')) {
          const std::string t = trim(line);
          if (t.empty()) continue;
          const auto sep = t.find(" - ");
          pk.push(Json::object({{"name", sep == std::string::npos ? t : t.substr(0, sep)},
                                {"description", sep == std::string::npos ? "" : t.substr(sep + 3)}}));
          if (pk.size() >= 100) break;
        }
        return Json::object({{"packages", pk}});
      });
  add(v, "pkg.update", "Refresh the package index", {"pkg.manage"}, "high", false, false, 300000, {"pkg_manage"},
      [](const Json&, ToolContext&) {
        const std::string m = pkg_manager();
        SandboxLimits lim;
        lim.timeout_ms = 290000;
        lim.cpu_seconds = 280;
        lim.mem_bytes = 2ull << 30;
        lim.allow_network = true;
        SandboxResult r = m == "apt-get" ? sandbox_exec("apt-get", {"update"}, "", lim)
                          : m == "dnf"   ? sandbox_exec("dnf", {"makecache"}, "", lim)
                                         : sandbox_exec("pacman", {"-Sy"}, "", lim);
        return Json::object({{"updated", r.success}, {"error", r.error}});
      });
  add(v, "pkg.list_installed", "Installed packages with versions", {"pkg.read"}, "low", true, false, 15000,
      {"pkg_read"}, [](const Json& in, ToolContext&) {
        Json pk = Json::array();
        const std::string filter = in.get_str("filter");
        if (have_cmd("dpkg-query")) {
          CmdResult r = sh({"dpkg-query", "-W", "-f=${Package} ${Version}\n"});
          for (auto& line : split(r.out, '\n')) {
            auto w = split_ws(line);
            if (w.size() < 2 || (!filter.empty() && !contains(w[0], filter))) continue;
            pk.push(Json::object({{"name", w[0]}, {"version", w[1]}}));
          }
        } else if (have_cmd("rpm")) {
          CmdResult r = sh({"rpm", "-qa", "--qf", "%{NAME} %{VERSION}\n"});
          for (auto& line : split(r.out, '\n')) {
            auto w = split_ws(line);
            if (w.size() >= 2) pk.push(Json::object({{"name", w[0]}, {"version", w[1]}}));
          }
        } else {
          tool_fail("no package database found");
        }
        return Json::object({{"packages", pk}, {"count", (int64_t)pk.size()}});
      });

  // ---------------------------------------------------------------------------------- monitor
  add(v, "monitor.cpu", "CPU utilisation, core count and load averages", {"monitor.read"}, "low", true, false, 5000,
      {"monitor_read"}, [](const Json& in, ToolContext&) {
        const double pct = cpu_percent((int)in.get_int("sample_ms", 200));
        Json la = Json::array();
        try {
          auto w = split_ws(read_file("/proc/loadavg"));
          for (int i = 0; i < 3 && i < (int)w.size(); ++i) la.push(std::stod(w[i]));
        } catch (...) {
        }
        return Json::object({{"percent", pct}, {"cores", (int64_t)sysconf(_SC_NPROCESSORS_ONLN)}, {"load_avg", la}});
      });
  add(v, "monitor.memory", "Memory total, used, available and utilisation percentage", {"monitor.read"}, "low", true,
      false, 5000, {"monitor_read"}, [](const Json&, ToolContext&) {
        auto m = meminfo();
        const double total = m["MemTotal"] / 1024.0, avail = m["MemAvailable"] / 1024.0;
        return Json::object({{"total_mb", total},
                             {"used_mb", total - avail},
                             {"available_mb", avail},
                             {"percent", total > 0 ? 100.0 * (total - avail) / total : 0.0}});
      });
  add(v, "monitor.disk", "Disk usage of a mount", {"monitor.read"}, "low", true, false, 5000, {"monitor_read"},
      [](const Json& in, ToolContext&) {
        const std::string p = in.get_str("path", "/");
        struct statvfs s;
        if (::statvfs(p.c_str(), &s) != 0) tool_fail("statvfs " + p + " failed");
        const double gb = 1024.0 * 1024.0 * 1024.0;
        const double total = (double)s.f_blocks * s.f_frsize / gb, avail = (double)s.f_bavail * s.f_frsize / gb;
        const double used = total - (double)s.f_bfree * s.f_frsize / gb;
        return Json::object({{"total_gb", total},
                             {"used_gb", used},
                             {"available_gb", avail},
                             {"percent", total > 0 ? 100.0 * used / total : 0.0}});
      });
  add(v, "monitor.network", "Interface byte / packet counters", {"monitor.read"}, "low", true, false, 5000,
      {"monitor_read"}, [](const Json& in, ToolContext&) { return net_dev(in.get_str("interface")); });
  add(v, "monitor.logs", "Recent system log lines", {"monitor.read"}, "low", true, false, 10000, {"monitor_read"},
      [](const Json& in, ToolContext&) {
        const int n = (int)std::max<int64_t>(1, std::min<int64_t>(1000, in.get_int("lines", 50)));
        const std::string svc = in.get_str("service");
        Json entries = Json::array();
        std::vector<std::string> lines;
        if (have_cmd("journalctl")) {
          std::vector<std::string> a{"journalctl", "-n", std::to_string(n), "--no-pager", "-o", "short-iso"};
          if (!svc.empty()) {
            a.push_back("-u");
            a.push_back(svc);
          }
          CmdResult r = sh(a, 8000);
          if (r.exit_code == 0) lines = split(r.out, '\n');
        }
        if (lines.empty()) {
          for (const char* f : {"/var/log/syslog", "/var/log/messages"}) {
            if (!file_exists(f)) continue;
            std::string data = read_file(f, 4 << 20);
            auto all = split(data, '\n');
            const size_t st = all.size() > (size_t)n + 1 ? all.size() - n - 1 : 0;
            lines.assign(all.begin() + st, all.end());
            break;
          }
        }
        for (auto& l : lines)
          if (!trim(l).empty() && (svc.empty() || contains(l, svc) || have_cmd("journalctl"))) entries.push(l);
        return Json::object({{"entries", entries}});
      });
  add(v, "monitor.ebpf_trace", "Process activity trace (syscall counters, open files, network connections) from /proc",
      {"monitor.read"}, "medium", true, false, 30000, {"monitor_read"}, [](const Json& in, ToolContext&) {
        const std::string type = in.get_str("trace_type", "syscalls");
        const int secs = (int)std::max<int64_t>(1, std::min<int64_t>(10, in.get_int("duration_secs", 1)));
        const int pid = (int)in.get_int("pid", 0);
        Json events = Json::array();
        if (type == "network") {
          for (const char* f : {"/proc/net/tcp", "/proc/net/tcp6"}) {
            std::ifstream inf(f);
            std::string line;
            std::getline(inf, line);
            while (std::getline(inf, line)) {
              auto w = split_ws(line);
              if (w.size() > 3) events.push(Json::object({{"local", w[1]}, {"remote", w[2]}, {"state", w[3]}}));
              if (events.size() > 500) break;
            }
          }
        } else if (type == "files") {
          const std::string fd = "/proc/" + (pid ? std::to_string(pid) : std::string("self")) + "/fd";
          if (DIR* d = ::opendir(fd.c_str())) {
            while (dirent* e = ::readdir(d)) {
              char buf[4096];
              const ssize_t n = ::readlink((fd + "/" + e->d_name).c_str(), buf, sizeof buf - 1);
              if (n > 0) events.push(std::string(buf, (size_t)n));
            }
            ::closedir(d);
          }
        } else {
          // per-process I/O syscall counters sampled over the window
          const std::string io = "/proc/" + (pid ? std::to_string(pid) : std::string("self")) + "/io";
          auto sample = [&]() {
            std::map<std::string, int64_t> m;
            try {
              for (auto& l : split(read_file(io), '\n')) {
                auto w = split_ws(l);
                if (w.size() == 2) m[w[0].substr(0, w[0].size() - 1)] = std::stoll(w[1]);
              }
            } catch (...) {
            }
            return m;
          };
          auto a = sample();
          std::this_thread::sleep_for(std::chrono::milliseconds(std::min(secs * 1000, 2000)));
          auto b = sample();
          for (auto& kv : b) events.push(Json::object({{"counter", kv.first}, {"delta", kv.second - a[kv.first]}}));
        }
        return Json::object({{"trace_type", type}, {"events", events}, {"duration_secs", secs}, {"method", "procfs"}});
      });
  add(v, "monitor.fs_watch", "Files changed under a path since a timestamp (mtime scan)", {"monitor.read"}, "low",
      true, false, 10000, {"monitor_read"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        const int64_t since = in.get_int("since_timestamp", now_unix() - 300);
        Json ev = Json::array();
        size_t budget = 20000;
        walk(p, in.get_bool("recursive", true) ? 6 : 0,
             [&](const std::string& f, const struct stat& st) {
               if (st.st_mtime >= since && ev.size() < 1000)
                 ev.push(Json::object({{"path", f},
                                       {"event", st.st_ctime >= since && st.st_ctime == st.st_mtime ? "modified" : "changed"},
                                       {"timestamp", (int64_t)st.st_mtime}}));
             },
             budget);
        return Json::object({{"path", p}, {"events", ev}, {"total_events", (int64_t)ev.size()}});
      });

  // ---------------------------------------------------------------------------------- hw
  add(v, "hw.info", "CPU, RAM, GPU and storage devices", {"hw.read"}, "low", true, false, 10000, {"hw_read"},
      [](const Json&, ToolContext&) {
        std::string cpu;
        try {
          for (auto& l : split(read_file("/proc/cpuinfo", 1 << 20), '\n'))
            if (starts_with(l, "model name")) {
              cpu = trim(l.substr(l.find(':') + 1));
              break;
            }
        } catch (...) {
        }
        auto m = meminfo();
        // GPUs: PCI display class devices; AMD Instinct / MI355X via the KFD topology
        Json gpus = Json::array();
        if (DIR* d = ::opendir("/sys/bus/pci/devices")) {
          while (dirent* e = ::readdir(d)) {
            const std::string base = std::string("/sys/bus/pci/devices/") + e->d_name;
            try {
              const std::string cls = trim(read_file(base + "/class", 32));
              if (!(starts_with(cls, "0x0300") || starts_with(cls, "0x0302") || starts_with(cls, "0x0380"))) continue;
              const std::string ven = trim(read_file(base + "/vendor", 32)), dev = trim(read_file(base + "/device", 32));
              const std::string vname = ven == "0x1002" ? "AMD" : ven == "0x10de" ? "NVIDIA" : ven == "0x8086" ? "Intel" : ven;
              gpus.push(Json::object({{"pci", std::string(e->d_name)}, {"vendor", vname}, {"device", dev}}));
            } catch (...) {
            }
          }
          ::closedir(d);
        }
        Json kfd = Json::array();
        if (DIR* d = ::opendir("/sys/class/kfd/kfd/topology/nodes")) {
          while (dirent* e = ::readdir(d)) {
            try {
              const std::string props =
                  read_file(std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name + "/properties", 1 << 16);
              for (auto& l : split(props, '\n'))
                if (starts_with(l, "gfx_target_version") && split_ws(l).size() > 1 && split_ws(l)[1] != "0")
                  kfd.push(Json::object({{"node", std::string(e->d_name)}, {"gfx_target_version", split_ws(l)[1]}}));
            } catch (...) {
            }
          }
          ::closedir(d);
        }
        std::string gpu = gpus.size() ? gpus[0].get_str("vendor") + " " + gpus[0].get_str("device") : "none";
        Json storage = Json::array();
        if (DIR* d = ::opendir("/sys/block")) {
          while (dirent* e = ::readdir(d)) {
            const std::string n = e->d_name;
            if (n[0] == '.' || starts_with(n, "loop") || starts_with(n, "ram")) continue;
            try {
              const double sectors = std::stod(read_file("/sys/block/" + n + "/size", 64));
              storage.push(Json::object({{"name", n}, {"size_gb", sectors * 512.0 / 1e9}}));
            } catch (...) {
            }
          }
          ::closedir(d);
        }
        return Json::object({{"cpu", cpu},
                             {"cores", (int64_t)sysconf(_SC_NPROCESSORS_ONLN)},
                             {"ram_mb", (int64_t)(m["MemTotal"] / 1024.0)},
                             {"gpu", gpu},
                             {"gpus", gpus},
                             {"amd_gpu_agents", kfd},
                             {"storage", storage}});
      });

  // ---------------------------------------------------------------------------------- sec
  add(v, "sec.check_perms", "Owner, group, mode and world-writability of a path", {"sec.read"}, "low", true, false,
      5000, {"sec_read"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        struct stat st;
        if (::stat(p.c_str(), &st) != 0) tool_fail("stat " + p + " failed");
        passwd* pw = getpwuid(st.st_uid);
        group* gr = getgrgid(st.st_gid);
        char mode[8];
        std::snprintf(mode, sizeof mode, "%o", (unsigned)(st.st_mode & 07777));
        return Json::object({{"owner", pw ? std::string(pw->pw_name) : std::to_string(st.st_uid)},
                             {"group", gr ? std::string(gr->gr_name) : std::to_string(st.st_gid)},
                             {"mode", std::string(mode)},
                             {"writable_by_others", (bool)(st.st_mode & S_IWOTH)}});
      });
  add(v, "sec.audit_query", "Query the tool audit ledger", {"sec.audit"}, "low", true, false, 5000, {"sec_read"},
      [](const Json& in, ToolContext& ctx) {
        return Json::object(
            {{"entries", ctx.svc->audit().query(in.get_str("tool_name"), "", "", "", (int)in.get_int("limit", 50))}});
      });
  add(v, "sec.grant", "Grant capabilities to an agent (optionally time-limited)", {"sec.admin"}, "critical", false,
      true, 5000, {"sec_manage"}, [](const Json& in, ToolContext& ctx) {
        const std::string agent = req_str(in, "agent_id");
        std::vector<std::string> caps;
        const auto& all = CapabilityChecker::all_capabilities();
        for (auto& c : in["capabilities"].as_arr()) {
          if (std::find(all.begin(), all.end(), c.as_str()) == all.end()) tool_fail("unknown capability: " + c.as_str());
          caps.push_back(c.as_str());
        }
        if (caps.empty()) tool_fail("no capabilities given");
        ctx.svc->caps().grant(agent, caps);
        const double hours = in.get_num("duration_hours", 0);
        const int64_t exp = hours > 0 ? now_unix() + (int64_t)(hours * 3600) : 0;
        Db db(ctx.paths->grants_db());
        db.exec("CREATE TABLE IF NOT EXISTS grants (agent_id TEXT, capability TEXT, reason TEXT, granted_at INTEGER, "
                "expires_at INTEGER)");
        for (auto& c : caps) {
          Stmt s(db, "INSERT INTO grants VALUES (?1,?2,?3,?4,?5)");
          s.bind(1, agent).bind(2, c).bind(3, in.get_str("reason")).bind(4, now_unix()).bind(5, exp).exec();
        }
        Json g = Json::array();
        for (auto& c : caps) g.push(c);
        return Json::object({{"success", true}, {"agent_id", agent}, {"granted", g},
                             {"expires_at", exp ? Json(rfc3339(exp)) : Json()}});
      });
  add(v, "sec.revoke", "Revoke capabilities from an agent", {"sec.admin"}, "critical", false, true, 5000,
      {"sec_manage"}, [](const Json& in, ToolContext& ctx) {
        const std::string agent = req_str(in, "agent_id");
        std::vector<std::string> caps;
        for (auto& c : in["capabilities"].as_arr()) caps.push_back(c.as_str());
        const int n = ctx.svc->caps().revoke(agent, caps, in.get_bool("revoke_all"));
        return Json::object({{"success", true}, {"agent_id", agent}, {"revoked_count", n}});
      });
  add(v, "sec.audit", "Audit log search by agent, tool and time window", {"sec.audit"}, "low", true, false, 5000,
      {"sec_read"}, [](const Json& in, ToolContext& ctx) {
        Json e = ctx.svc->audit().query(in.get_str("tool_name"), in.get_str("agent_id"), in.get_str("since"),
                                        in.get_str("until"), (int)in.get_int("limit", 100));
        return Json::object({{"entries", e}, {"total", (int64_t)e.size()}, {"chain_valid", ctx.svc->audit().verify_chain()}});
      });
  add(v, "sec.scan", "Security scan: world-writable /etc files, SUID binaries, listening ports, weak permissions",
      {"sec.read"}, "medium", true, false, 30000, {"sec_read"}, [](const Json& in, ToolContext&) {
        std::set<std::string> checks;
        for (auto& c : in["checks"].as_arr()) checks.insert(c.as_str());
        auto want = [&](const char* c) { return checks.empty() || checks.count(c); };
        Json findings = Json::array();
        int high = 0, med = 0;
        size_t budget = 50000;
        if (want("world_writable")) {
          walk("/etc", 3,
               [&](const std::string& p, const struct stat& st) {
                 if (!S_ISLNK(st.st_mode) && (st.st_mode & S_IWOTH) && findings.size() < 200) {
                   findings.push(Json::object({{"check", "world_writable"}, {"severity", "high"}, {"path", p}}));
                   ++high;
                 }
               },
               budget);
        }
        if (want("suid")) {
          static const std::set<std::string> expected = {"sudo", "su", "passwd", "mount", "umount", "ping", "chsh",
                                                         "chfn", "newgrp", "gpasswd", "pkexec", "fusermount", "fusermount3"};
          for (const char* dir : {"/usr/bin", "/usr/sbin", "/bin", "/sbin"}) {
            walk(dir, 0,
                 [&](const std::string& p, const struct stat& st) {
                   if (S_ISREG(st.st_mode) && (st.st_mode & S_ISUID)) {
                     const std::string base = p.substr(p.rfind('/') + 1);
                     if (!expected.count(base)) {
                       findings.push(Json::object({{"check", "suid"}, {"severity", "medium"}, {"path", p}}));
                       ++med;
                     }
                   }
                 },
                 budget);
          }
        }
        if (want("ports")) {
          for (int p : listening_ports()) {
            const bool risky = p == 23 || p == 21 || p == 3389 || p == 5900;
            findings.push(Json::object({{"check", "listening_port"}, {"severity", risky ? "high" : "info"}, {"port", p}}));
            if (risky) ++high;
          }
        }
        if (want("permissions")) {
          for (const char* f : {"/etc/shadow", "/etc/gshadow", "/etc/sudoers"}) {
            struct stat st;
            if (::stat(f, &st) == 0 && (st.st_mode & (S_IROTH | S_IWOTH))) {
              findings.push(Json::object({{"check", "weak_permissions"}, {"severity", "high"}, {"path", f}}));
              ++high;
            }
          }
        }
        return Json::object({{"findings", findings},
                             {"total_findings", (int64_t)findings.size()},
                             {"risk_level", risk_from(high, med)}});
      });
  add(v, "sec.cert_generate", "Generate a self-signed CA and a service certificate", {"sec.admin", "fs_write"}, "high",
      false, true, 10000, {"sec_manage"}, [](const Json& in, ToolContext& ctx) {
        const std::string svc = req_str(in, "service_name");
        static const std::regex re("^[A-Za-z0-9_-]{1,64}$");
        if (!std::regex_match(svc, re)) tool_fail("invalid service name");
        return gen_certs(svc, in.get_str("cert_dir", ctx.paths->data_dir + "/certs"), (int)in.get_int("validity_years", 1));
      });
  add(v, "sec.cert_rotate", "Back up and regenerate a service certificate", {"sec.admin", "fs_write", "service_manage"},
      "high", false, true, 30000, {"sec_manage"}, [](const Json& in, ToolContext& ctx) {
        const std::string svc = req_str(in, "service_name");
        static const std::regex re("^[A-Za-z0-9_-]{1,64}$");
        if (!std::regex_match(svc, re)) tool_fail("invalid service name");
        const std::string dir = in.get_str("cert_dir", ctx.paths->data_dir + "/certs");
        bool backed = false;
        const std::string stamp = std::to_string(now_unix());
        for (const char* ext : {".crt", ".key"}) {
          const std::string f = dir + "/" + svc + ext;
          if (file_exists(f) && ::rename(f.c_str(), (f + ".bak." + stamp).c_str()) == 0) backed = true;
        }
        Json g = gen_certs(svc, dir, 1);
        return Json::object({{"success", g.get_bool("success")}, {"backed_up", backed}, {"regenerated", true},
                             {"service_name", svc}});
      });
  add(v, "sec.file_integrity", "SHA-256 file integrity baseline / check", {"sec.read"}, "medium", true, false, 30000,
      {"sec_read"}, [](const Json& in, ToolContext& ctx) {
        const std::string mode = in.get_str("mode", "check");
        std::vector<std::string> paths;
        for (auto& p : in["paths"].as_arr()) paths.push_back(p.as_str());
        if (paths.empty()) paths = {"/etc/passwd", "/etc/group", "/etc/hosts", "/etc/ssh/sshd_config"};
        std::vector<std::string> files;
        for (auto& p : paths) {
          struct stat st;
          if (::stat(p.c_str(), &st) != 0) {
            files.push_back(p);  // reported as missing in check mode
            continue;
          }
          if (S_ISDIR(st.st_mode)) {
            size_t budget = 5000;
            walk(p, 4, [&](const std::string& f, const struct stat& s2) { if (S_ISREG(s2.st_mode)) files.push_back(f); },
                 budget);
          } else {
            files.push_back(p);
          }
        }
        Db& db = integrity_db(ctx);
        std::lock_guard<std::recursive_mutex> g(db.mutex());
        Json modified = Json::array(), added = Json::array(), missing = Json::array();
        int checked = 0;
        for (auto& f : files) {
          std::string h;
          bool exists = true;
          try {
            h = sha256_hex(read_file(f, 64 << 20));
          } catch (...) {
            exists = false;
          }
          ++checked;
          Stmt q(db, "SELECT sha256 FROM baseline WHERE path = ?1");
          q.bind(1, f);
          const bool known = q.step();
          const std::string old = known ? q.col_text(0) : "";
          if (mode == "baseline") {
            if (!exists) continue;
            Stmt s(db, "INSERT OR REPLACE INTO baseline VALUES (?1,?2,?3,?4)");
            s.bind(1, f).bind(2, h).bind(3, (int64_t)0).bind(4, now_unix()).exec();
          } else {
            if (!exists && known) missing.push(f);
            else if (exists && !known) added.push(f);
            else if (exists && known && old != h) modified.push(f);
          }
        }
        return Json::object({{"mode", mode}, {"checked", checked}, {"modified", modified}, {"new_files", added},
                             {"missing_files", missing}});
      });
  add(v, "sec.scan_rootkits", "Rootkit indicators: hidden processes, executables in /dev/shm and /tmp, known paths",
      {"sec.read"}, "medium", true, false, 30000, {"sec_read"}, [](const Json&, ToolContext&) {
        Json findings = Json::array();
        // executables / scripts in world-writable scratch dirs
        size_t budget = 20000;
        for (const char* d : {"/dev/shm", "/tmp", "/var/tmp"}) {
          walk(d, 2,
               [&](const std::string& p, const struct stat& st) {
                 if (S_ISREG(st.st_mode) && (st.st_mode & 0111) && findings.size() < 200)
                   findings.push(Json::object({{"check", "executable_in_scratch"}, {"path", p}}));
               },
               budget);
        }
        // known rootkit artefacts
        for (const char* p : {"/dev/.udev/rules.d", "/usr/lib/libproc.a", "/etc/ld.so.hash", "/usr/bin/.sshd",
                              "/dev/.lib", "/usr/share/.aPa"})
          if (file_exists(p)) findings.push(Json::object({{"check", "known_artefact"}, {"path", std::string(p)}}));
        // deleted-binary processes (a classic in-memory implant indicator)
        if (DIR* d = ::opendir("/proc")) {
          while (dirent* e = ::readdir(d)) {
            if (!isdigit((unsigned char)e->d_name[0])) continue;
            char buf[4096];
            const ssize_t n = ::readlink((std::string("/proc/") + e->d_name + "/exe").c_str(), buf, sizeof buf - 1);
            if (n > 0 && ends_with(std::string(buf, (size_t)n), " (deleted)"))
              findings.push(Json::object({{"check", "deleted_executable"}, {"pid", std::atoi(e->d_name)},
                                          {"exe", std::string(buf, (size_t)n)}}));
          }
          ::closedir(d);
        }
        return Json::object({{"findings", findings}, {"total_findings", (int64_t)findings.size()},
                             {"clean", findings.size() == 0}});
      });
}

}  // namespace aiosn
