// Host utilities shared by the native control-plane cores: SQLite (declared against the system
// libsqlite3.so.0 ABI -- no dev headers in the image), SHA-256 (OpenSSL libcrypto), UUIDs, time,
// and a no-shell subprocess runner with time / output limits.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace aiosn {

// ------------------------------------------------------------------------------------ SQLite
struct sqlite3_;
struct sqlite3_stmt_;

class Db;
class Stmt {
 public:
  Stmt(Db& db, const std::string& sql);
  ~Stmt();
  Stmt(const Stmt&) = delete;
  Stmt& operator=(const Stmt&) = delete;
  Stmt& bind(int idx, const std::string& v);
  Stmt& bind(int idx, int64_t v);
  Stmt& bind(int idx, double v);
  Stmt& bind_blob(int idx, const void* p, size_t n);
  Stmt& bind_null(int idx);
  bool step();  // true while a row is available
  void exec();  // run to completion
  void reset();
  int64_t col_int(int c) const;
  double col_double(int c) const;
  std::string col_text(int c) const;
  std::string col_blob(int c) const;
  bool col_null(int c) const;

 private:
  Db& db_;
  sqlite3_stmt_* st_ = nullptr;
};

class Db {
 public:
  explicit Db(const std::string& path);  // ":memory:" supported; parent dirs created
  ~Db();
  Db(const Db&) = delete;
  Db& operator=(const Db&) = delete;
  void exec(const std::string& sql);
  int64_t last_insert_rowid() const;
  int changes() const;
  std::string errmsg() const;
  sqlite3_* handle() { return db_; }
  std::recursive_mutex& mutex() { return mu_; }
  const std::string& path() const { return path_; }

 private:
  sqlite3_* db_ = nullptr;
  std::string path_;
  std::recursive_mutex mu_;
};

// ------------------------------------------------------------------------------------ misc
std::string sha256_hex(const std::string& data);
std::string uuid4();
int64_t now_unix();
int64_t now_ms();
std::string now_rfc3339();
std::string rfc3339(int64_t unix_seconds);
void mkdirs(const std::string& dir);
std::string env_or(const char* name, const std::string& def);
std::string read_file(const std::string& path, size_t max_bytes = (size_t)-1);
bool file_exists(const std::string& path);
std::string trim(const std::string& s);
std::string lower(std::string s);
std::vector<std::string> split(const std::string& s, char sep);
std::vector<std::string> split_ws(const std::string& s);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
bool contains(const std::string& s, const std::string& p);
bool icontains(const std::string& s, const std::string& p);

// ------------------------------------------------------------------------------------ processes
struct CmdResult {
  int exit_code = -1;   // -1: could not start
  bool timed_out = false;
  std::string out, err;
};
struct CmdLimits {
  int timeout_ms = 30000;
  size_t max_output = 1 << 20;
  // sandbox (tools/sandbox.rs semantics); 0 = unlimited
  size_t mem_bytes = 0;
  int cpu_seconds = 0;
  int max_fds = 0;
  int max_procs = 0;
  bool clear_env = false;
  std::vector<std::string> env;   // KEY=VALUE added after clearing
  std::string cwd;
  std::string stdin_data;
};
// argv[0] is looked up in PATH; never goes through a shell
CmdResult run_cmd(const std::vector<std::string>& argv, const CmdLimits& lim = CmdLimits());
bool have_cmd(const std::string& name);

}  // namespace aiosn
