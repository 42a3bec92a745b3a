// fs (13), process (6) and service (5) tools.  I/O contracts follow the reference handlers
// (tools/src/{fs,process,service}/*.rs; SURVEY §2.4 per-tool table); Linux only.
#include <dirent.h>
#include <fnmatch.h>
#include <grp.h>
#include <pwd.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <fstream>

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

std::string errno_msg(const std::string& what, const std::string& path) {
  return what + " " + path + ": " + std::strerror(errno);
}

std::string file_type(mode_t m) {
  if (S_ISDIR(m)) return "directory";
  if (S_ISLNK(m)) return "symlink";
  if (S_ISREG(m)) return "file";
  return "other";
}

std::string mode_str(mode_t m) {
  char b[8];
  std::snprintf(b, sizeof b, "%o", (unsigned)(m & 07777));
  return b;
}

void remove_tree(const std::string& p) {
  struct stat st;
  if (::lstat(p.c_str(), &st) != 0) return;
  if (S_ISDIR(st.st_mode)) {
    if (DIR* d = ::opendir(p.c_str())) {
      while (dirent* e = ::readdir(d)) {
        const std::string n = e->d_name;
        if (n == "." || n == "..") continue;
        remove_tree(p + "/" + n);
      }
      ::closedir(d);
    }
    if (::rmdir(p.c_str()) != 0) tool_fail(errno_msg("rmdir", p));
  } else if (::unlink(p.c_str()) != 0) {
    tool_fail(errno_msg("unlink", p));
  }
}

void copy_tree(const std::string& src, const std::string& dst) {
  struct stat st;
  if (::lstat(src.c_str(), &st) != 0) tool_fail(errno_msg("stat", src));
  if (S_ISDIR(st.st_mode)) {
    ::mkdir(dst.c_str(), st.st_mode & 07777);
    DIR* d = ::opendir(src.c_str());
    if (!d) tool_fail(errno_msg("opendir", src));
    while (dirent* e = ::readdir(d)) {
      const std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      copy_tree(src + "/" + n, dst + "/" + n);
    }
    ::closedir(d);
  } else if (S_ISLNK(st.st_mode)) {
    char buf[4096];
    const ssize_t n = ::readlink(src.c_str(), buf, sizeof buf - 1);
    if (n < 0) tool_fail(errno_msg("readlink", src));
    buf[n] = 0;
    if (::symlink(buf, dst.c_str()) != 0) tool_fail(errno_msg("symlink", dst));
  } else {
    std::ifstream in(src, std::ios::binary);
    std::ofstream out(dst, std::ios::binary | std::ios::trunc);
    if (!in || !out) tool_fail("copy " + src + " -> " + dst + " failed");
    out << in.rdbuf();
    ::chmod(dst.c_str(), st.st_mode & 07777);
  }
}

void search_dir(const std::string& dir, const std::string& pat, int depth, int max_depth, Json& out, size_t cap) {
  if (depth > max_depth || out.size() >= cap) return;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return;
  while (dirent* e = ::readdir(d)) {
    const std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    const std::string p = dir == "/" ? "/" + n : dir + "/" + n;
    if (fnmatch(pat.c_str(), n.c_str(), 0) == 0) out.push(p);
    if (out.size() >= cap) break;
    struct stat st;
    if (::lstat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) search_dir(p, pat, depth + 1, max_depth, out, cap);
  }
  ::closedir(d);
}

// ----------------------------------------------------------------------------- /proc helpers
struct ProcInfo {
  int pid = 0;
  std::string name, state, cmdline;
  double cpu = 0, mem_mb = 0;
  int threads = 0;
  int64_t started = 0;
};

double uptime_s() {
  try {
    return std::stod(read_file("/proc/uptime"));
  } catch (...) {
    return 0;
  }
}

bool read_proc(int pid, ProcInfo& pi) {
  std::string stat;
  try {
    stat = read_file("/proc/" + std::to_string(pid) + "/stat");
  } catch (...) {
    return false;
  }
  const auto l = stat.find('('), r = stat.rfind(')');
  if (l == std::string::npos || r == std::string::npos) return false;
  pi.pid = pid;
  pi.name = stat.substr(l + 1, r - l - 1);
  auto f = split_ws(stat.substr(r + 2));  // fields from #3 (state)
  if (f.size() < 22) return false;
  pi.state = f[0];
  const double hz = (double)sysconf(_SC_CLK_TCK);
  const double ut = std::stod(f[11]), st = std::stod(f[12]);
  const double start = std::stod(f[19]) / hz;
  pi.threads = std::stoi(f[17]);
  const double up = uptime_s();
  const double life = up - start;
  pi.cpu = life > 0 ? 100.0 * (ut + st) / hz / life : 0;
  const double rss_pages = std::stod(f[21]);
  pi.mem_mb = rss_pages * (double)sysconf(_SC_PAGESIZE) / (1024.0 * 1024.0);
  pi.started = now_unix() - (int64_t)life;
  try {
    std::string c = read_file("/proc/" + std::to_string(pid) + "/cmdline", 8192);
    for (auto& ch : c)
      if (ch == 0) ch = ' ';
    pi.cmdline = trim(c);
  } catch (...) {
  }
  return true;
}

int parse_signal(const Json& v) {
  if (v.is_num()) return (int)v.as_int();
  std::string s = v.str_or("SIGTERM");
  if (!s.empty() && isdigit((unsigned char)s[0])) return std::stoi(s);
  if (!starts_with(s, "SIG")) s = "SIG" + s;
  static const std::pair<const char*, int> names[] = {
      {"SIGHUP", SIGHUP},   {"SIGINT", SIGINT},   {"SIGQUIT", SIGQUIT}, {"SIGKILL", SIGKILL}, {"SIGTERM", SIGTERM},
      {"SIGUSR1", SIGUSR1}, {"SIGUSR2", SIGUSR2}, {"SIGSTOP", SIGSTOP}, {"SIGCONT", SIGCONT}};
  for (auto& n : names)
    if (s == n.first) return n.second;
  tool_fail("unknown signal: " + s);
}

void guard_pid(int pid) {
  if (pid <= 1) tool_fail("refusing to signal pid " + std::to_string(pid));
  if (pid == (int)getpid()) tool_fail("refusing to signal the tool service itself");
}

std::string systemctl_prop(const std::string& unit, const std::string& prop) {
  CmdLimits l;
  l.timeout_ms = 5000;
  CmdResult r = run_cmd({"systemctl", "show", unit, "--property=" + prop, "--value"}, l);
  return trim(r.out);
}

Json service_status(const std::string& name) {
  if (!have_cmd("systemctl")) tool_fail("systemctl not available");
  const std::string unit = ends_with(name, ".service") ? name : name + ".service";
  Json o = Json::object();
  o.set("name", name);
  o.set("status", systemctl_prop(unit, "ActiveState"));
  const std::string pid = systemctl_prop(unit, "MainPID");
  o.set("pid", (int64_t)(pid.empty() ? 0 : std::stoll(pid)));
  o.set("uptime", systemctl_prop(unit, "ActiveEnterTimestamp"));
  return o;
}

Json systemctl_action(const std::string& action, const std::string& name) {
  if (!have_cmd("systemctl")) tool_fail("systemctl not available");
  CmdLimits l;
  l.timeout_ms = 30000;
  CmdResult r = run_cmd({"systemctl", action, name}, l);
  if (r.exit_code != 0) tool_fail("systemctl " + action + " " + name + " failed: " + trim(r.err));
  return service_status(name);
}

}  // namespace

void add_fs_process_service_tools(std::vector<ToolSpec>& v) {
  // ---------------------------------------------------------------------------------- fs
  add(v, "fs.read", "Read a file's content", {"fs.read"}, "low", true, false, 5000, {"fs_read"},
      [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        struct stat st;
        if (::stat(p.c_str(), &st) != 0) tool_fail(errno_msg("stat", p));
        if (S_ISDIR(st.st_mode)) tool_fail(p + " is a directory");
        const size_t cap = (size_t)in.get_int("max_bytes", 10 << 20);
        std::string c = read_file(p, cap);
        return Json::object({{"content", c}, {"size", (int64_t)st.st_size}});
      });
  add(v, "fs.write", "Write content to a file (creating parent directories)", {"fs.write"}, "medium", false, true,
      10000, {"fs_write"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        const std::string c = in.get_str("content");
        const auto slash = p.rfind('/');
        if (slash > 0) mkdirs(p.substr(0, slash));
        std::ofstream f(p, std::ios::binary | (in.get_bool("append") ? std::ios::app : std::ios::trunc));
        if (!f) tool_fail(errno_msg("open", p));
        f << c;
        if (!f) tool_fail(errno_msg("write", p));
        return Json::object({{"bytes_written", (int64_t)c.size()}});
      });
  add(v, "fs.delete", "Delete a file or directory", {"fs.delete"}, "high", false, false, 10000,
      {"fs_write", "fs_delete"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        if (p == "/" || p == "/etc" || p == "/usr" || p == "/bin" || p == "/boot") tool_fail("refusing to delete " + p);
        struct stat st;
        if (::lstat(p.c_str(), &st) != 0) tool_fail(errno_msg("stat", p));
        if (S_ISDIR(st.st_mode)) {
          if (in.get_bool("recursive")) remove_tree(p);
          else if (::rmdir(p.c_str()) != 0) tool_fail(errno_msg("rmdir", p));
        } else if (::unlink(p.c_str()) != 0) {
          tool_fail(errno_msg("unlink", p));
        }
        return Json::object({{"deleted", true}});
      });
  add(v, "fs.list", "List a directory with entry type, size and last-modified time", {"fs.read"}, "low", true, false,
      5000, {"fs_read"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        DIR* d = ::opendir(p.c_str());
        if (!d) tool_fail(errno_msg("opendir", p));
        Json entries = Json::array();
        while (dirent* e = ::readdir(d)) {
          const std::string n = e->d_name;
          if (n == "." || n == "..") continue;
          struct stat st;
          const std::string fp = p == "/" ? "/" + n : p + "/" + n;
          if (::lstat(fp.c_str(), &st) != 0) continue;
          entries.push(Json::object({{"name", n},
                                     {"type", file_type(st.st_mode)},
                                     {"size", (int64_t)st.st_size},
                                     {"modified", rfc3339(st.st_mtime)}}));
        }
        ::closedir(d);
        return Json::object({{"entries", entries}});
      });
  add(v, "fs.stat", "File metadata: size, permissions, timestamps and type flags", {"fs.read"}, "low", true, false,
      5000, {"fs_read"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        struct stat st, lst;
        if (::lstat(p.c_str(), &lst) != 0) tool_fail(errno_msg("stat", p));
        if (::stat(p.c_str(), &st) != 0) st = lst;
        return Json::object({{"size", (int64_t)st.st_size},
                             {"permissions", mode_str(st.st_mode)},
                             {"modified", rfc3339(st.st_mtime)},
                             {"accessed", rfc3339(st.st_atime)},
                             {"is_dir", (bool)S_ISDIR(st.st_mode)},
                             {"is_file", (bool)S_ISREG(st.st_mode)},
                             {"is_symlink", (bool)S_ISLNK(lst.st_mode)},
                             {"uid", (int64_t)st.st_uid},
                             {"gid", (int64_t)st.st_gid}});
      });
  add(v, "fs.mkdir", "Create a directory", {"fs.write"}, "low", true, true, 5000, {"fs_write"},
      [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        if (in.get_bool("recursive", true)) mkdirs(p);
        else if (::mkdir(p.c_str(), 0755) != 0 && errno != EEXIST) tool_fail(errno_msg("mkdir", p));
        struct stat st;
        if (::stat(p.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) tool_fail("mkdir " + p + " failed");
        return Json::object({{"created", true}});
      });
  add(v, "fs.move", "Move or rename a file or directory", {"fs.write", "fs.delete"}, "medium", false, true, 10000,
      {"fs_write"}, [](const Json& in, ToolContext&) {
        const std::string s = abs_path(in, "source"), d = abs_path(in, "destination");
        if (::rename(s.c_str(), d.c_str()) != 0) {
          if (errno != EXDEV) tool_fail(errno_msg("rename", s));
          copy_tree(s, d);
          remove_tree(s);
        }
        return Json::object({{"moved", true}});
      });
  add(v, "fs.copy", "Copy a file or directory tree", {"fs.read", "fs.write"}, "medium", false, true, 30000,
      {"fs_write"}, [](const Json& in, ToolContext&) {
        copy_tree(abs_path(in, "source"), abs_path(in, "destination"));
        return Json::object({{"copied", true}});
      });
  add(v, "fs.chmod", "Change permission bits (octal mode string)", {"fs.write"}, "high", true, true, 5000,
      {"fs_write", "fs_permissions"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        const std::string m = in.get_str("mode");
        if (m.empty()) tool_fail("missing required field 'mode'");
        const mode_t mode = (mode_t)std::stoul(m, nullptr, 8);
        if (::chmod(p.c_str(), mode) != 0) tool_fail(errno_msg("chmod", p));
        return Json::object({{"changed", true}});
      });
  add(v, "fs.chown", "Change file owner/group", {"fs.admin"}, "critical", true, true, 5000,
      {"fs_write", "fs_permissions"}, [](const Json& in, ToolContext&) {
        const std::string p = abs_path(in, "path");
        const int uid = (int)in.get_int("uid", -1), gid = (int)in.get_int("gid", -1);
        if (::chown(p.c_str(), (uid_t)uid, (gid_t)gid) != 0) tool_fail(errno_msg("chown", p));
        return Json::object({{"changed", true}});
      });
  add(v, "fs.symlink", "Create a symbolic link", {"fs.write"}, "medium", false, true, 5000, {"fs_write"},
      [](const Json& in, ToolContext&) {
        const std::string t = abs_path(in, "target"), l = abs_path(in, "link");
        if (::symlink(t.c_str(), l.c_str()) != 0) tool_fail(errno_msg("symlink", l));
        return Json::object({{"created", true}});
      });
  add(v, "fs.search", "Find files by glob pattern under a directory", {"fs.read"}, "low", true, false, 30000,
      {"fs_read"}, [](const Json& in, ToolContext&) {
        const std::string d = abs_path(in, "directory");
        Json m = Json::array();
        search_dir(d, in.get_str("pattern", "*"), 1, (int)in.get_int("max_depth", 5), m,
                   (size_t)in.get_int("max_results", 1000));
        return Json::object({{"matches", m}});
      });
  add(v, "fs.disk_usage", "Filesystem capacity and usage for a path", {"fs.read"}, "low", true, false, 5000,
      {"fs_read"}, [](const Json& in, ToolContext&) {
        const std::string p = in.get_str("path", "/");
        struct statvfs s;
        if (::statvfs(p.c_str(), &s) != 0) tool_fail(errno_msg("statvfs", p));
        const double total = (double)s.f_blocks * s.f_frsize, avail = (double)s.f_bavail * s.f_frsize;
        const double used = total - (double)s.f_bfree * s.f_frsize;
        return Json::object({{"total_bytes", (int64_t)total},
                             {"used_bytes", (int64_t)used},
                             {"available_bytes", (int64_t)avail},
                             {"usage_percent", total > 0 ? 100.0 * used / total : 0.0}});
      });

  // ---------------------------------------------------------------------------------- process
  add(v, "process.list", "List processes with pid, name, cpu, memory and status", {"process.read"}, "low", true,
      false, 10000, {"process_read"}, [](const Json& in, ToolContext&) {
        Json ps = Json::array();
        DIR* d = ::opendir("/proc");
        const std::string filter = in.get_str("name");
        const size_t cap = (size_t)in.get_int("limit", 500);
        while (d && ps.size() < cap) {
          dirent* e = ::readdir(d);
          if (!e) break;
          if (!isdigit((unsigned char)e->d_name[0])) continue;
          ProcInfo pi;
          if (!read_proc(std::atoi(e->d_name), pi)) continue;
          if (!filter.empty() && !icontains(pi.name, filter)) continue;
          ps.push(Json::object({{"pid", pi.pid},
                                {"name", pi.name},
                                {"cpu", pi.cpu},
                                {"memory", pi.mem_mb},
                                {"status", pi.state}}));
        }
        if (d) ::closedir(d);
        return Json::object({{"processes", ps}});
      });
  add(v, "process.spawn", "Start a detached process with arguments and environment variables", {"process.execute"},
      "high", false, false, 30000, {"process_manage"}, [](const Json& in, ToolContext&) {
        const std::string cmd = req_str(in, "command");
        std::vector<std::string> argv{cmd};
        for (auto& a : in["args"].as_arr()) argv.push_back(a.is_str() ? a.as_str() : a.dump());
        std::vector<std::pair<std::string, std::string>> env;
        for (auto& kv : in["env"].as_obj()) env.emplace_back(kv.first, kv.second.str_or(kv.second.dump()));
        int pfd[2];
        if (pipe(pfd) != 0) tool_fail("pipe failed");
        const pid_t pid = fork();
        if (pid < 0) tool_fail("fork failed");
        if (pid == 0) {
          setsid();
          const pid_t g = fork();  // double fork: the child is re-parented, never a zombie here
          if (g != 0) {
            ::write(pfd[1], &g, sizeof g);
            _exit(0);
          }
          ::close(pfd[0]);
          ::close(pfd[1]);
          for (auto& kv : env) setenv(kv.first.c_str(), kv.second.c_str(), 1);
          std::vector<char*> args;
          for (auto& a : argv) args.push_back(const_cast<char*>(a.c_str()));
          args.push_back(nullptr);
          execvp(args[0], args.data());
          _exit(127);
        }
        ::close(pfd[1]);
        pid_t g = -1;
        ::read(pfd[0], &g, sizeof g);
        ::close(pfd[0]);
        int st;
        waitpid(pid, &st, 0);
        return Json::object({{"pid", (int64_t)g}});
      });
  add(v, "process.kill", "Terminate a process", {"process.kill"}, "critical", false, false, 5000, {"process_manage"},
      [](const Json& in, ToolContext&) {
        const int pid = (int)in.get_int("pid", 0);
        guard_pid(pid);
        const int sig = in.has("signal") ? parse_signal(in["signal"]) : SIGTERM;
        if (::kill(pid, sig) != 0) tool_fail(errno_msg("kill", std::to_string(pid)));
        return Json::object({{"killed", true}});
      });
  add(v, "process.info", "Details of one process", {"process.read"}, "low", true, false, 5000, {"process_read"},
      [](const Json& in, ToolContext&) {
        ProcInfo pi;
        const int pid = (int)in.get_int("pid", 0);
        if (!read_proc(pid, pi)) tool_fail("no such process: " + std::to_string(pid));
        return Json::object({{"pid", pi.pid},
                             {"name", pi.name},
                             {"cmdline", pi.cmdline},
                             {"cpu", pi.cpu},
                             {"memory", pi.mem_mb},
                             {"threads", pi.threads},
                             {"started_at", rfc3339(pi.started)}});
      });
  add(v, "process.signal", "Send a signal to a process", {"process.signal"}, "high", false, false, 5000,
      {"process_manage"}, [](const Json& in, ToolContext&) {
        const int pid = (int)in.get_int("pid", 0);
        guard_pid(pid);
        if (::kill(pid, parse_signal(in["signal"])) != 0) tool_fail(errno_msg("kill", std::to_string(pid)));
        return Json::object({{"sent", true}});
      });
  add(v, "process.cgroup", "Manage cgroup v2 groups: create, add a pid, set CPU/memory/IO limits, info, delete",
      {"process.admin"}, "high", false, true, 10000, {"process_manage"}, [](const Json& in, ToolContext&) {
        const std::string action = req_str(in, "action"), group = req_str(in, "group_name");
        if (group.find('/') != std::string::npos || group.find("..") != std::string::npos)
          tool_fail("invalid group name");
        const std::string root = env_or("AIOS_CGROUP_ROOT", "/sys/fs/cgroup/aios");
        const std::string dir = root + "/" + group;
        Json details = Json::object();
        auto wr = [&](const std::string& f, const std::string& val) {
          std::ofstream o(dir + "/" + f);
          if (!o) tool_fail("cannot write " + dir + "/" + f);
          o << val;
          details.set(f, val);
        };
        if (action == "create") {
          mkdirs(dir);
          if (!file_exists(dir)) tool_fail("cannot create cgroup " + dir);
        } else if (action == "add") {
          wr("cgroup.procs", std::to_string(in.get_int("pid", 0)));
        } else if (action == "set") {
          if (in.has("cpu_weight")) wr("cpu.weight", std::to_string(in.get_int("cpu_weight")));
          if (in.has("memory_max_mb")) wr("memory.max", std::to_string(in.get_int("memory_max_mb") << 20));
          if (in.has("io_weight")) wr("io.weight", "default " + std::to_string(in.get_int("io_weight")));
        } else if (action == "info") {
          for (const char* f : {"cgroup.procs", "cpu.weight", "memory.max", "memory.current", "io.weight"}) {
            try {
              details.set(f, trim(read_file(dir + "/" + f, 65536)));
            } catch (...) {
            }
          }
        } else if (action == "delete") {
          if (::rmdir(dir.c_str()) != 0) tool_fail(errno_msg("rmdir", dir));
        } else {
          tool_fail("unknown action: " + action);
        }
        return Json::object({{"success", true}, {"action", action}, {"group_name", group}, {"details", details}});
      });

  // ---------------------------------------------------------------------------------- service
  add(v, "service.list", "List systemd services with status and pid", {"service.read"}, "low", true, false, 10000,
      {"service_read"}, [](const Json&, ToolContext&) {
        if (!have_cmd("systemctl")) tool_fail("systemctl not available");
        CmdLimits l;
        l.timeout_ms = 10000;
        CmdResult r = run_cmd({"systemctl", "list-units", "--type=service", "--all", "--no-pager", "--plain",
                               "--no-legend"}, l);
        Json svcs = Json::array();
        for (auto& line : split(r.out, '\n')) {
          auto f = split_ws(line);
          if (f.size() < 4) continue;
          std::string name = f[0];
          if (ends_with(name, ".service")) name = name.substr(0, name.size() - 8);
          svcs.push(Json::object({{"name", name}, {"status", f[2] + "/" + f[3]}, {"pid", 0}}));
        }
        return Json::object({{"services", svcs}});
      });
  add(v, "service.start", "Start a service", {"service.manage"}, "high", false, true, 15000, {"service_manage"},
      [](const Json& in, ToolContext&) {
        Json s = systemctl_action("start", req_str(in, "name"));
        return Json::object({{"started", true}, {"pid", s["pid"]}});
      });
  add(v, "service.stop", "Stop a service", {"service.manage"}, "high", false, true, 15000, {"service_manage"},
      [](const Json& in, ToolContext&) {
        systemctl_action("stop", req_str(in, "name"));
        return Json::object({{"stopped", true}});
      });
  add(v, "service.restart", "Restart a service", {"service.manage"}, "high", false, true, 30000, {"service_manage"},
      [](const Json& in, ToolContext&) {
        Json s = systemctl_action("restart", req_str(in, "name"));
        return Json::object({{"restarted", true}, {"pid", s["pid"]}});
      });
  add(v, "service.status", "Status of a service", {"service.read"}, "low", true, false, 5000, {"service_read"},
      [](const Json& in, ToolContext&) { return service_status(req_str(in, "name")); });
}

}  // namespace aiosn
