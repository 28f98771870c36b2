// JSON parser and value accessors (see json.h). Serialisation lives in json_dump.cpp.
#include "json.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace dfs {

namespace {

const Json kNull;
const std::string kEmpty;
const Json::Array kEmptyArray;
const Json::Object kEmptyObject;

// Recursive-descent parser over [p, end).
struct Parser {
  const char* p;
  const char* end;
  int depth = 0;

  [[noreturn]] void fail(const char* what) const { throw std::runtime_error(std::string("json: ") + what); }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if (static_cast<size_t>(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void utf8(uint32_t cp, std::string& out) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    if (end - p < 4) fail("short unicode escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad unicode escape");
    }
    return v;
  }
  std::string string();
  Json number();
  Json value();
};

std::string Parser::string() {
  if (p >= end || *p != '"') fail("expected string");
  ++p;
  std::string out;
  for (;;) {
    const char* q = p;
    while (q < end && *q != '"' && *q != '\\') ++q;
    out.append(p, q);
    p = q;
    if (p >= end) fail("unterminated string");
    if (*p == '"') {
      ++p;
      return out;
    }
    ++p;  // the escape character
    if (p >= end) fail("bad escape");
    char c = *p++;
    switch (c) {
      case '"': out.push_back('"'); break;
      case '\\': out.push_back('\\'); break;
      case '/': out.push_back('/'); break;
      case 'b': out.push_back('\b'); break;
      case 'f': out.push_back('\f'); break;
      case 'n': out.push_back('\n'); break;
      case 'r': out.push_back('\r'); break;
      case 't': out.push_back('\t'); break;
      case 'u': {
        uint32_t cp = hex4();
        if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
          const char* save = p;
          p += 2;
          uint32_t lo = hex4();
          if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          else p = save;
        }
        utf8(cp, out);
        break;
      }
      default: fail("bad escape");
    }
  }
}

Json Parser::number() {
  const char* s = p;
  bool is_float = false;
  if (p < end && *p == '-') ++p;
  while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) {
    if (*p == '.' || *p == 'e' || *p == 'E') is_float = true;
    ++p;
  }
  std::string tok(s, p);
  if (tok.empty() || tok == "-") fail("bad number");
  char* e = nullptr;
  if (!is_float) {
    errno = 0;
    long long v = std::strtoll(tok.c_str(), &e, 10);
    if (errno == 0 && e && *e == 0) return Json(static_cast<int64_t>(v));
    errno = 0;
    unsigned long long u = std::strtoull(tok.c_str(), &e, 10);  // u64 above INT64_MAX
    if (errno == 0 && e && *e == 0 && tok[0] != '-') return Json(static_cast<uint64_t>(u));
  }
  double d = std::strtod(tok.c_str(), &e);
  if (!e || *e != 0) fail("bad number");
  return Json(d);
}

Json Parser::value() {
  ws();
  if (p >= end) fail("unexpected end");
  char c = *p;
  if (c == '{' || c == '[') {
    if (++depth > 512) fail("nesting too deep");
    ++p;
    bool obj = c == '{';
    char close = obj ? '}' : ']';
    Json::Object o;
    Json::Array a;
    ws();
    if (p < end && *p == close) {
      ++p;
    } else {
      for (;;) {
        if (obj) {
          ws();
          std::string k = string();
          ws();
          if (p >= end || *p != ':') fail("expected ':'");
          ++p;
          o.emplace_back(std::move(k), value());
        } else {
          a.push_back(value());
        }
        ws();
        if (p < end && *p == ',') {
          ++p;
          continue;
        }
        if (p < end && *p == close) {
          ++p;
          break;
        }
        fail("expected ',' or a closing bracket");
      }
    }
    --depth;
    return obj ? Json(std::move(o)) : Json(std::move(a));
  }
  if (c == '"') return Json(string());
  if (lit("true")) return Json(true);
  if (lit("false")) return Json(false);
  if (lit("null")) return Json();
  if (lit("NaN")) return Json(std::nan(""));
  if (lit("Infinity")) return Json(HUGE_VAL);
  if (lit("-Infinity")) return Json(-HUGE_VAL);
  return number();
}

}  // namespace

Json Json::parse(const char* p, size_t n) {
  Parser ps{p, p + n};
  Json v = ps.value();
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing characters");
  return v;
}

Json Json::parse(const std::string& text) { return parse(text.data(), text.size()); }

const std::string& Json::as_string() const { return t_ == Type::String ? s_ : kEmpty; }

size_t Json::size() const {
  if (t_ == Type::Array) return a_->size();
  if (t_ == Type::Object) return o_->size();
  return 0;
}

void Json::own() {
  if (t_ == Type::Array && a_.use_count() > 1) a_ = std::make_shared<Array>(*a_);
  if (t_ == Type::Object && o_.use_count() > 1) o_ = std::make_shared<Object>(*o_);
}

const Json& Json::operator[](size_t i) const {
  if (t_ != Type::Array || i >= a_->size()) return kNull;
  return (*a_)[i];
}

void Json::push_back(Json v) {
  if (t_ == Type::Null) *this = Json(Array{});
  if (t_ != Type::Array) throw std::runtime_error("json: push_back on non-array");
  own();
  a_->push_back(std::move(v));
}

const Json::Array& Json::items() const { return t_ == Type::Array ? *a_ : kEmptyArray; }

Json::Array& Json::items() {
  if (t_ == Type::Null) *this = Json(Array{});
  if (t_ != Type::Array) throw std::runtime_error("json: not an array");
  own();
  return *a_;
}

const Json* Json::find(const std::string& key) const {
  if (t_ != Type::Object) return nullptr;
  for (auto& kv : *o_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

Json* Json::find(const std::string& key) {
  if (t_ != Type::Object) return nullptr;
  own();
  for (auto& kv : *o_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

const Json& Json::operator[](const std::string& key) const {
  const Json* v = find(key);
  return v ? *v : kNull;
}

Json& Json::set(const std::string& key, Json v) {
  if (t_ == Type::Null) *this = Json(Object{});
  if (t_ != Type::Object) throw std::runtime_error("json: set on non-object");
  own();
  for (auto& kv : *o_)
    if (kv.first == key) {
      kv.second = std::move(v);
      return kv.second;
    }
  o_->emplace_back(key, std::move(v));
  return o_->back().second;
}

bool Json::erase(const std::string& key) {
  if (t_ != Type::Object) return false;
  own();
  for (auto it = o_->begin(); it != o_->end(); ++it)
    if (it->first == key) {
      o_->erase(it);
      return true;
    }
  return false;
}

const Json::Object& Json::fields() const { return t_ == Type::Object ? *o_ : kEmptyObject; }

Json::Object& Json::fields() {
  if (t_ == Type::Null) *this = Json(Object{});
  if (t_ != Type::Object) throw std::runtime_error("json: not an object");
  own();
  return *o_;
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (t_ == Type::Int && o.t_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (t_ != o.t_) return false;
  switch (t_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: {
      if (o_->size() != o.o_->size()) return false;
      for (auto& kv : *o_) {
        const Json* v = o.find(kv.first);
        if (!v || *v != kv.second) return false;
      }
      return true;
    }
    default: return false;
  }
}

}  // namespace dfs
