#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace aiosn {

const Json& Json::null_ref() {
  static const Json n;
  return n;
}

double Json::str_to_num(const std::string& s, double d) {
  if (s.empty()) return d;
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  return (end && *end == 0) ? v : d;
}

const Json& Json::operator[](const std::string& k) const {
  if (t_ != OBJ) return null_ref();
  for (auto& p : *o_)
    if (p.first == k) return p.second;
  return null_ref();
}

bool Json::has(const std::string& k) const {
  if (t_ != OBJ) return false;
  for (auto& p : *o_)
    if (p.first == k) return true;
  return false;
}

Json& Json::set(const std::string& k, Json v) {
  if (t_ != OBJ) {
    *this = object();
  }
  // copy-on-write: values share storage after a copy
  if (o_.use_count() > 1) o_ = std::make_shared<Obj>(*o_);
  for (auto& p : *o_)
    if (p.first == k) {
      p.second = std::move(v);
      return p.second;
    }
  o_->emplace_back(k, std::move(v));
  return o_->back().second;
}

Json& Json::push(Json v) {
  if (t_ != ARR) *this = array();
  if (a_.use_count() > 1) a_ = std::make_shared<Arr>(*a_);
  a_->push_back(std::move(v));
  return a_->back();
}

std::string Json::get_str(const std::string& k, const std::string& d) const {
  const Json& v = (*this)[k];
  if (v.is_str()) return v.s_;
  if (v.is_num()) return v.dump();
  if (v.is_bool()) return v.b_ ? "true" : "false";
  return d;
}
int64_t Json::get_int(const std::string& k, int64_t d) const {
  const Json& v = (*this)[k];
  return (v.is_num() || v.is_str()) ? v.as_int(d) : d;
}
double Json::get_num(const std::string& k, double d) const {
  const Json& v = (*this)[k];
  return (v.is_num() || v.is_str()) ? v.as_num(d) : d;
}
bool Json::get_bool(const std::string& k, bool d) const {
  const Json& v = (*this)[k];
  if (v.is_bool()) return v.b_;
  if (v.is_num()) return v.n_ != 0;
  if (v.is_str()) return v.s_ == "true" || v.s_ == "1" || v.s_ == "yes";
  return d;
}

bool Json::operator==(const Json& o) const {
  if (t_ != o.t_) return false;
  switch (t_) {
    case NUL: return true;
    case BOOL: return b_ == o.b_;
    case NUM: return n_ == o.n_;
    case STR: return s_ == o.s_;
    case ARR: return *a_ == *o.a_;
    case OBJ: {
      if (o_->size() != o.o_->size()) return false;
      for (auto& p : *o_)
        if (!(o[p.first] == p.second) || !o.has(p.first)) return false;
      return true;
    }
  }
  return false;
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent < 0) return;
    out += '\n';
    out.append((size_t)indent * d, ' ');
  };
  switch (t_) {
    case NUL: out += "null"; break;
    case BOOL: out += b_ ? "true" : "false"; break;
    case NUM: {
      if (int_) {
        out += std::to_string(i_);
      } else if (!std::isfinite(n_)) {
        out += "null";
      } else if (n_ == std::floor(n_) && std::fabs(n_) < 1e15) {
        out += std::to_string((int64_t)n_);
        out += ".0";
      } else {
        char buf[32];
        std::snprintf(buf, sizeof buf, "%.17g", n_);
        // shortest round-trip-ish: trim to 15 significant digits when exact
        char buf2[32];
        std::snprintf(buf2, sizeof buf2, "%.15g", n_);
        out += (std::strtod(buf2, nullptr) == n_) ? buf2 : buf;
      }
    } break;
    case STR:
      out += '"';
      out += json_escape(s_);
      out += '"';
      break;
    case ARR: {
      out += '[';
      for (size_t i = 0; i < a_->size(); ++i) {
        if (i) out += indent < 0 ? ", " : ",";
        nl(depth + 1);
        (*a_)[i].dump_to(out, indent, depth + 1);
      }
      if (!a_->empty()) nl(depth);
      out += ']';
    } break;
    case OBJ: {
      out += '{';
      size_t i = 0;
      for (auto& p : *o_) {
        if (i++) out += indent < 0 ? ", " : ",";
        nl(depth + 1);
        out += '"';
        out += json_escape(p.first);
        out += "\": ";
        p.second.dump_to(out, indent, depth + 1);
      }
      if (!o_->empty()) nl(depth);
      out += '}';
    } break;
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

namespace {
struct Parser {
  const std::string& s;
  size_t i = 0;
  int depth = 0;
  explicit Parser(const std::string& src) : s(src) {}
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      const char c = s[i++];
      if (c == '"') break;
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
        const char e = s[i++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              i += 2;
              const uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            utf8(out, cp);
          } break;
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    return out;
  }
  Json num() {
    const size_t st = i;
    bool integral = true;
    if (s[i] == '-') ++i;
    while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
    if (i < s.size() && s[i] == '.') {
      integral = false;
      ++i;
      while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      integral = false;
      ++i;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
      while (i < s.size() && isdigit((unsigned char)s[i])) ++i;
    }
    const std::string tok = s.substr(st, i - st);
    if (tok.empty() || tok == "-") fail("bad number");
    if (integral && tok.size() < 19) return Json((int64_t)std::strtoll(tok.c_str(), nullptr, 10));
    return Json(std::strtod(tok.c_str(), nullptr));
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    if (++depth > 512) fail("nesting too deep");
    Json out;
    const char c = s[i];
    if (c == '{') {
      ++i;
      out = Json::object();
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
      } else {
        while (true) {
          ws();
          std::string k = str();
          ws();
          if (i >= s.size() || s[i] != ':') fail("expected ':'");
          ++i;
          out.set(k, value());
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == '}') { ++i; break; }
          fail("expected ',' or '}'");
        }
      }
    } else if (c == '[') {
      ++i;
      out = Json::array();
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
      } else {
        while (true) {
          out.push(value());
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == ']') { ++i; break; }
          fail("expected ',' or ']'");
        }
      }
    } else if (c == '"') {
      out = Json(str());
    } else if (c == 't' && s.compare(i, 4, "true") == 0) {
      i += 4;
      out = Json(true);
    } else if (c == 'f' && s.compare(i, 5, "false") == 0) {
      i += 5;
      out = Json(false);
    } else if (c == 'n' && s.compare(i, 4, "null") == 0) {
      i += 4;
    } else if (c == '-' || isdigit((unsigned char)c)) {
      out = num();
    } else {
      fail("unexpected character");
    }
    --depth;
    return out;
  }
};
}  // namespace

Json Json::parse(const std::string& s) {
  Parser p(s);
  Json v = p.value();
  p.ws();
  if (p.i != s.size()) p.fail("trailing characters");
  return v;
}

bool Json::try_parse(const std::string& s, Json& out) {
  try {
    out = parse(s);
    return true;
  } catch (const std::exception&) {
    return false;
  }
}

}  // namespace aiosn
