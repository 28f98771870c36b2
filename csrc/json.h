// Minimal JSON value for the metadata plane: Raft log entries, snapshots, state-machine
// commands and their results, and the HTTP/JSON Raft peer protocol. The command and
// snapshot encodings follow the reference's serde externally-tagged layout, e.g.
// {"Master":{"CreateFile":{"path":...}}} (reference: dfs/metaserver/src/simple_raft.rs:56-68,
// 254-389).
//
// Objects keep insertion order (what Python's json module and serde both do) in a
// vector; lookups are linear, which is the right trade for the small objects of a
// command. Large maps (a shard's whole namespace) never live in a Json value on the hot
// path: the state machines keep typed C++ structures and only build Json for snapshots.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace dfs {

class Json {
 public:
  enum class Type : uint8_t { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::vector<std::pair<std::string, Json>>;

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : t_(Type::Bool), b_(b) {}
  Json(int v) : t_(Type::Int), i_(v) {}
  Json(int64_t v) : t_(Type::Int), i_(v) {}
  Json(uint64_t v) : t_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(uint32_t v) : t_(Type::Int), i_(v) {}
  Json(double v) : t_(Type::Double), d_(v) {}
  Json(const char* s) : t_(Type::String), s_(s) {}
  Json(std::string s) : t_(Type::String), s_(std::move(s)) {}
  Json(Array a) : t_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : t_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json array() { return Json(Array{}); }
  static Json object() { return Json(Object{}); }
  // Throws std::runtime_error on malformed input.
  static Json parse(const std::string& text);
  static Json parse(const char* p, size_t n);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::Double; }
  bool is_int() const { return t_ == Type::Int; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return t_ == Type::Bool ? b_ : (t_ == Type::Int ? i_ != 0 : dflt); }
  int64_t as_int(int64_t dflt = 0) const {
    return t_ == Type::Int ? i_ : (t_ == Type::Double ? static_cast<int64_t>(d_) : (t_ == Type::Bool ? b_ : dflt));
  }
  uint64_t as_u64(uint64_t dflt = 0) const { return static_cast<uint64_t>(as_int(static_cast<int64_t>(dflt))); }
  double as_double(double dflt = 0) const {
    return t_ == Type::Double ? d_ : (t_ == Type::Int ? static_cast<double>(i_) : dflt);
  }
  const std::string& as_string() const;
  std::string str(const std::string& dflt = "") const { return t_ == Type::String ? s_ : dflt; }

  // Arrays
  size_t size() const;
  const Json& operator[](size_t i) const;
  const Json& operator[](int i) const { return (*this)[static_cast<size_t>(i)]; }
  void push_back(Json v);
  const Array& items() const;
  Array& items();

  // Objects
  const Json* find(const std::string& key) const;
  Json* find(const std::string& key);
  bool has(const std::string& key) const { return find(key) != nullptr; }
  // Missing keys read as null (never throws), so optional fields need no checks.
  const Json& operator[](const std::string& key) const;
  const Json& operator[](const char* key) const { return (*this)[std::string(key)]; }
  Json& set(const std::string& key, Json v);  // insert or replace, keeps position
  bool erase(const std::string& key);
  const Object& fields() const;
  Object& fields();

  std::string dump() const;
  void dump_to(std::string& out) const;

  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void own();  // copy-on-write for shared containers
  Type t_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

void json_escape(const std::string& s, std::string& out);

}  // namespace dfs
