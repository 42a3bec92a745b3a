#include "util.h"

#include <fcntl.h>
#include <openssl/sha.h>
#include <poll.h>
#include <signal.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <random>
#include <sstream>

// The SQLite C API subset used here (stable ABI of libsqlite3.so.0; the image ships the library
// but not sqlite3.h).
extern "C" {
struct sqlite3;
struct sqlite3_stmt;
int sqlite3_open_v2(const char*, sqlite3**, int, const char*);
int sqlite3_close_v2(sqlite3*);
int sqlite3_exec(sqlite3*, const char*, int (*)(void*, int, char**, char**), void*, char**);
void sqlite3_free(void*);
const char* sqlite3_errmsg(sqlite3*);
int sqlite3_prepare_v2(sqlite3*, const char*, int, sqlite3_stmt**, const char**);
int sqlite3_bind_text(sqlite3_stmt*, int, const char*, int, void (*)(void*));
int sqlite3_bind_int64(sqlite3_stmt*, int, long long);
int sqlite3_bind_double(sqlite3_stmt*, int, double);
int sqlite3_bind_blob(sqlite3_stmt*, int, const void*, int, void (*)(void*));
int sqlite3_bind_null(sqlite3_stmt*, int);
int sqlite3_step(sqlite3_stmt*);
int sqlite3_reset(sqlite3_stmt*);
int sqlite3_finalize(sqlite3_stmt*);
long long sqlite3_column_int64(sqlite3_stmt*, int);
double sqlite3_column_double(sqlite3_stmt*, int);
const unsigned char* sqlite3_column_text(sqlite3_stmt*, int);
const void* sqlite3_column_blob(sqlite3_stmt*, int);
int sqlite3_column_bytes(sqlite3_stmt*, int);
int sqlite3_column_type(sqlite3_stmt*, int);
long long sqlite3_last_insert_rowid(sqlite3*);
int sqlite3_changes(sqlite3*);
int sqlite3_busy_timeout(sqlite3*, int);
}

namespace aiosn {

namespace {
constexpr int SQLITE_OK = 0, SQLITE_ROW = 100, SQLITE_DONE = 101, SQLITE_NULL = 5;
constexpr int SQLITE_OPEN_READWRITE = 0x2, SQLITE_OPEN_CREATE = 0x4, SQLITE_OPEN_FULLMUTEX = 0x10000,
              SQLITE_OPEN_URI = 0x40;
void (*const SQLITE_TRANSIENT)(void*) = reinterpret_cast<void (*)(void*)>(-1);
inline sqlite3* H(sqlite3_* p) { return reinterpret_cast<sqlite3*>(p); }
inline sqlite3_stmt* S(sqlite3_stmt_* p) { return reinterpret_cast<sqlite3_stmt*>(p); }
}  // namespace

Db::Db(const std::string& path) : path_(path) {
  if (path != ":memory:") {
    const auto slash = path.rfind('/');
    if (slash != std::string::npos && slash > 0) mkdirs(path.substr(0, slash));
  }
  sqlite3* h = nullptr;
  const int rc = sqlite3_open_v2(path.c_str(), &h, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE | SQLITE_OPEN_FULLMUTEX |
                                                      SQLITE_OPEN_URI, nullptr);
  if (rc != SQLITE_OK) {
    std::string msg = h ? sqlite3_errmsg(h) : "out of memory";
    if (h) sqlite3_close_v2(h);
    throw std::runtime_error("sqlite open " + path + ": " + msg);
  }
  db_ = reinterpret_cast<sqlite3_*>(h);
  sqlite3_busy_timeout(h, 5000);
  if (path != ":memory:") exec("PRAGMA journal_mode=WAL; PRAGMA synchronous=NORMAL;");
}

Db::~Db() {
  if (db_) sqlite3_close_v2(H(db_));
}

void Db::exec(const std::string& sql) {
  std::lock_guard<std::recursive_mutex> g(mu_);
  char* err = nullptr;
  if (sqlite3_exec(H(db_), sql.c_str(), nullptr, nullptr, &err) != SQLITE_OK) {
    std::string msg = err ? err : "?";
    sqlite3_free(err);
    throw std::runtime_error("sqlite: " + msg + " in: " + sql.substr(0, 200));
  }
}
int64_t Db::last_insert_rowid() const { return sqlite3_last_insert_rowid(H(db_)); }
int Db::changes() const { return sqlite3_changes(H(db_)); }
std::string Db::errmsg() const { return sqlite3_errmsg(H(db_)); }

Stmt::Stmt(Db& db, const std::string& sql) : db_(db) {
  sqlite3_stmt* st = nullptr;
  if (sqlite3_prepare_v2(H(db.handle()), sql.c_str(), -1, &st, nullptr) != SQLITE_OK)
    throw std::runtime_error("sqlite prepare: " + db.errmsg() + " in: " + sql.substr(0, 200));
  st_ = reinterpret_cast<sqlite3_stmt_*>(st);
}
Stmt::~Stmt() {
  if (st_) sqlite3_finalize(S(st_));
}
Stmt& Stmt::bind(int idx, const std::string& v) {
  sqlite3_bind_text(S(st_), idx, v.data(), (int)v.size(), SQLITE_TRANSIENT);
  return *this;
}
Stmt& Stmt::bind(int idx, int64_t v) {
  sqlite3_bind_int64(S(st_), idx, v);
  return *this;
}
Stmt& Stmt::bind(int idx, double v) {
  sqlite3_bind_double(S(st_), idx, v);
  return *this;
}
Stmt& Stmt::bind_blob(int idx, const void* p, size_t n) {
  sqlite3_bind_blob(S(st_), idx, p, (int)n, SQLITE_TRANSIENT);
  return *this;
}
Stmt& Stmt::bind_null(int idx) {
  sqlite3_bind_null(S(st_), idx);
  return *this;
}
bool Stmt::step() {
  const int rc = sqlite3_step(S(st_));
  if (rc == SQLITE_ROW) return true;
  if (rc == SQLITE_DONE) return false;
  throw std::runtime_error("sqlite step: " + db_.errmsg());
}
void Stmt::exec() {
  while (step()) {
  }
}
void Stmt::reset() { sqlite3_reset(S(st_)); }
int64_t Stmt::col_int(int c) const { return sqlite3_column_int64(S(st_), c); }
double Stmt::col_double(int c) const { return sqlite3_column_double(S(st_), c); }
std::string Stmt::col_text(int c) const {
  const unsigned char* t = sqlite3_column_text(S(st_), c);
  return t ? std::string((const char*)t, sqlite3_column_bytes(S(st_), c)) : std::string();
}
std::string Stmt::col_blob(int c) const {
  const void* p = sqlite3_column_blob(S(st_), c);
  return p ? std::string((const char*)p, sqlite3_column_bytes(S(st_), c)) : std::string();
}
bool Stmt::col_null(int c) const { return sqlite3_column_type(S(st_), c) == SQLITE_NULL; }

// ------------------------------------------------------------------------------------ misc
std::string sha256_hex(const std::string& data) {
  unsigned char md[SHA256_DIGEST_LENGTH];
  SHA256(reinterpret_cast<const unsigned char*>(data.data()), data.size(), md);
  static const char* hx = "0123456789abcdef";
  std::string out(2 * SHA256_DIGEST_LENGTH, '0');
  for (int i = 0; i < SHA256_DIGEST_LENGTH; ++i) {
    out[2 * i] = hx[md[i] >> 4];
    out[2 * i + 1] = hx[md[i] & 15];
  }
  return out;
}

std::string uuid4() {
  static thread_local std::mt19937_64 rng(std::random_device{}() ^ (uint64_t)now_ms());
  uint64_t a = rng(), b = rng();
  a = (a & 0xFFFFFFFFFFFF0FFFULL) | 0x0000000000004000ULL;
  b = (b & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
  char buf[40];
  std::snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xFFFF),
                (unsigned)(a & 0xFFFF), (unsigned)(b >> 48), (unsigned long long)(b & 0xFFFFFFFFFFFFULL));
  return buf;
}

int64_t now_unix() { return (int64_t)std::time(nullptr); }
int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
std::string rfc3339(int64_t t) {
  std::time_t tt = (std::time_t)t;
  std::tm tm{};
  gmtime_r(&tt, &tm);
  char buf[40];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S+00:00", &tm);
  return buf;
}
std::string now_rfc3339() {
  const int64_t ms = now_ms();
  std::time_t tt = (std::time_t)(ms / 1000);
  std::tm tm{};
  gmtime_r(&tt, &tm);
  char buf[48];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  char out[64];
  std::snprintf(out, sizeof out, "%s.%03d+00:00", buf, (int)(ms % 1000));
  return out;
}

void mkdirs(const std::string& dir) {
  if (dir.empty()) return;
  std::string cur;
  for (size_t i = 0; i < dir.size(); ++i) {
    cur += dir[i];
    if ((dir[i] == '/' && i > 0) || i + 1 == dir.size()) ::mkdir(cur.c_str(), 0755);
  }
}

std::string env_or(const char* name, const std::string& def) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::string(v) : def;
}

std::string read_file(const std::string& path, size_t max_bytes) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string out;
  char buf[65536];
  while (f && out.size() < max_bytes) {
    f.read(buf, (std::streamsize)std::min(sizeof buf, max_bytes - out.size()));
    out.append(buf, (size_t)f.gcount());
  }
  return out;
}

bool file_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}
std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}
std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}
std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> out;
  std::istringstream is(s);
  std::string w;
  while (is >> w) out.push_back(w);
  return out;
}
bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}
bool contains(const std::string& s, const std::string& p) { return s.find(p) != std::string::npos; }
bool icontains(const std::string& s, const std::string& p) { return lower(s).find(lower(p)) != std::string::npos; }

// ------------------------------------------------------------------------------------ processes
bool have_cmd(const std::string& name) {
  if (name.find('/') != std::string::npos) return ::access(name.c_str(), X_OK) == 0;
  const std::string path = env_or("PATH", "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin");
  for (auto& d : split(path, ':'))
    if (!d.empty() && ::access((d + "/" + name).c_str(), X_OK) == 0) return true;
  return false;
}

CmdResult run_cmd(const std::vector<std::string>& argv, const CmdLimits& lim) {
  CmdResult r;
  if (argv.empty()) return r;
  int po[2], pe[2], pi[2];
  if (pipe2(po, O_CLOEXEC) || pipe2(pe, O_CLOEXEC) || pipe2(pi, O_CLOEXEC)) {
    r.err = "pipe failed";
    return r;
  }
  std::vector<char*> args;
  for (auto& a : argv) args.push_back(const_cast<char*>(a.c_str()));
  args.push_back(nullptr);
  std::vector<std::string> envs;
  std::vector<char*> envp;
  if (lim.clear_env) {
    envs.push_back("PATH=/usr/bin:/bin");
    for (auto& e : lim.env) envs.push_back(e);
    for (auto& e : envs) envp.push_back(const_cast<char*>(e.c_str()));
    envp.push_back(nullptr);
  }
  const pid_t pid = fork();
  if (pid < 0) {
    r.err = "fork failed";
    return r;
  }
  if (pid == 0) {
    setpgid(0, 0);
    dup2(pi[0], 0);
    dup2(po[1], 1);
    dup2(pe[1], 2);
    if (!lim.cwd.empty() && chdir(lim.cwd.c_str()) != 0) _exit(126);
    auto lim1 = [](int res, rlim_t v) {
      struct rlimit rl{v, v};
      setrlimit(res, &rl);
    };
    if (lim.mem_bytes) lim1(RLIMIT_AS, (rlim_t)lim.mem_bytes);
    if (lim.cpu_seconds) lim1(RLIMIT_CPU, (rlim_t)lim.cpu_seconds);
    if (lim.max_fds) lim1(RLIMIT_NOFILE, (rlim_t)lim.max_fds);
    if (lim.max_procs) lim1(RLIMIT_NPROC, (rlim_t)lim.max_procs);
    if (lim.clear_env) execvpe(args[0], args.data(), envp.data());
    else execvp(args[0], args.data());
    _exit(127);
  }
  ::close(po[1]);
  ::close(pe[1]);
  ::close(pi[0]);
  if (!lim.stdin_data.empty()) {
    size_t off = 0;
    while (off < lim.stdin_data.size()) {
      const ssize_t n = ::write(pi[1], lim.stdin_data.data() + off, lim.stdin_data.size() - off);
      if (n <= 0) break;
      off += (size_t)n;
    }
  }
  ::close(pi[1]);
  const int64_t deadline = now_ms() + lim.timeout_ms;
  struct pollfd fds[2] = {{po[0], POLLIN, 0}, {pe[0], POLLIN, 0}};
  int open_fds = 2;
  char buf[16384];
  while (open_fds > 0) {
    const int64_t left = deadline - now_ms();
    if (left <= 0) {
      r.timed_out = true;
      kill(-pid, SIGKILL);
      break;
    }
    if (poll(fds, 2, (int)std::min<int64_t>(left, 200)) < 0) break;
    for (int k = 0; k < 2; ++k) {
      if (fds[k].fd < 0) continue;
      if (fds[k].revents & (POLLIN | POLLHUP | POLLERR)) {
        const ssize_t n = ::read(fds[k].fd, buf, sizeof buf);
        if (n <= 0) {
          ::close(fds[k].fd);
          fds[k].fd = -1;
          --open_fds;
        } else {
          std::string& dst = k == 0 ? r.out : r.err;
          if (dst.size() < lim.max_output) dst.append(buf, std::min((size_t)n, lim.max_output - dst.size()));
        }
      }
    }
  }
  for (auto& f : fds)
    if (f.fd >= 0) ::close(f.fd);
  int status = 0;
  if (r.timed_out) {
    waitpid(pid, &status, 0);
    r.exit_code = -1;
  } else {
    // the pipes closed; reap (bounded by the deadline)
    while (true) {
      const pid_t w = waitpid(pid, &status, WNOHANG);
      if (w == pid) break;
      if (now_ms() > deadline) {
        kill(-pid, SIGKILL);
        waitpid(pid, &status, 0);
        r.timed_out = true;
        break;
      }
      usleep(2000);
    }
    if (!r.timed_out) r.exit_code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
  }
  if (r.exit_code == 127 && r.out.empty() && r.err.empty()) r.err = "command not found: " + argv[0];
  return r;
}

}  // namespace aiosn
