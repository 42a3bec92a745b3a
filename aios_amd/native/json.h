// Minimal JSON value + parser/serializer for the native control-plane cores (tool I/O is JSON
// bytes, LLM outputs are parsed for JSON plans).  Objects keep insertion order, numbers keep an
// "integral" flag so ids/sizes round-trip as integers.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace aiosn {

class Json {
 public:
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ };
  using Arr = std::vector<Json>;
  using Obj = std::vector<std::pair<std::string, Json>>;

  Json() : t_(NUL) {}
  Json(std::nullptr_t) : t_(NUL) {}
  Json(bool b) : t_(BOOL), b_(b) {}
  Json(int v) : t_(NUM), n_((double)v), i_(v), int_(true) {}
  Json(int64_t v) : t_(NUM), n_((double)v), i_(v), int_(true) {}
  Json(uint64_t v) : t_(NUM), n_((double)v), i_((int64_t)v), int_(true) {}
  Json(long long v) : t_(NUM), n_((double)v), i_((int64_t)v), int_(true) {}
  Json(unsigned v) : t_(NUM), n_((double)v), i_(v), int_(true) {}
  Json(double v) : t_(NUM), n_(v), i_((int64_t)v), int_(false) {}
  Json(const char* s) : t_(STR), s_(s) {}
  Json(const std::string& s) : t_(STR), s_(s) {}
  Json(std::string&& s) : t_(STR), s_(std::move(s)) {}
  Json(const Arr& a) : t_(ARR), a_(std::make_shared<Arr>(a)) {}
  Json(Arr&& a) : t_(ARR), a_(std::make_shared<Arr>(std::move(a))) {}
  static Json object() {
    Json j;
    j.t_ = OBJ;
    j.o_ = std::make_shared<Obj>();
    return j;
  }
  static Json array() {
    Json j;
    j.t_ = ARR;
    j.a_ = std::make_shared<Arr>();
    return j;
  }
  static Json object(std::initializer_list<std::pair<const char*, Json>> kv) {
    Json j = object();
    for (auto& p : kv) j.set(p.first, p.second);
    return j;
  }

  Type type() const { return t_; }
  bool is_null() const { return t_ == NUL; }
  bool is_bool() const { return t_ == BOOL; }
  bool is_num() const { return t_ == NUM; }
  bool is_str() const { return t_ == STR; }
  bool is_arr() const { return t_ == ARR; }
  bool is_obj() const { return t_ == OBJ; }

  bool as_bool(bool d = false) const { return t_ == BOOL ? b_ : (t_ == NUM ? n_ != 0 : d); }
  double as_num(double d = 0) const { return t_ == NUM ? n_ : (t_ == STR ? str_to_num(s_, d) : d); }
  int64_t as_int(int64_t d = 0) const {
    if (t_ == NUM) return int_ ? i_ : (int64_t)n_;
    if (t_ == STR) return (int64_t)str_to_num(s_, (double)d);
    return d;
  }
  const std::string& as_str() const {
    static const std::string empty;
    return t_ == STR ? s_ : empty;
  }
  std::string str_or(const std::string& d) const { return t_ == STR ? s_ : d; }
  const Arr& as_arr() const {
    static const Arr empty;
    return t_ == ARR ? *a_ : empty;
  }
  const Obj& as_obj() const {
    static const Obj empty;
    return t_ == OBJ ? *o_ : empty;
  }
  size_t size() const { return t_ == ARR ? a_->size() : (t_ == OBJ ? o_->size() : 0); }

  // object access
  const Json& operator[](const std::string& k) const;
  bool has(const std::string& k) const;
  Json& set(const std::string& k, Json v);
  // convenience getters with defaults
  std::string get_str(const std::string& k, const std::string& d = "") const;
  int64_t get_int(const std::string& k, int64_t d = 0) const;
  double get_num(const std::string& k, double d = 0) const;
  bool get_bool(const std::string& k, bool d = false) const;

  // array access
  const Json& operator[](size_t i) const { return (t_ == ARR && i < a_->size()) ? (*a_)[i] : null_ref(); }
  Json& push(Json v);

  std::string dump(int indent = -1) const;
  static Json parse(const std::string& s);            // throws std::runtime_error
  static bool try_parse(const std::string& s, Json& out);

  bool operator==(const Json& o) const;

 private:
  static const Json& null_ref();
  static double str_to_num(const std::string& s, double d);
  void dump_to(std::string& out, int indent, int depth) const;

  Type t_;
  bool b_ = false;
  double n_ = 0;
  int64_t i_ = 0;
  bool int_ = false;
  std::string s_;
  std::shared_ptr<Arr> a_;
  std::shared_ptr<Obj> o_;
};

std::string json_escape(const std::string& s);

}  // namespace aiosn
