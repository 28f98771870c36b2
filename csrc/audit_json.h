// Python-compatible JSON text for the S3 audit log (C56/C59): the record's canonical form
// (audit.py::canonical_json: reference field order, compact separators, non-ASCII kept as
// UTF-8) and its HMAC-SHA256, shared by the native logger (audit_log.cpp) and the native
// audit_reader (tools/audit_reader.cpp), so both hash byte-identically to the Python side.
#pragma once
#include <openssl/hmac.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "json.h"

namespace dfs {
namespace audit {

inline const char* const kFields[] = {"timestamp",   "timestamp_ms", "request_id",  "remote_ip", "user_id",
                               "role_arn",    "action",       "resource",    "status_code", "error_code",
                               "user_agent",  "duration_ms",  "previous_hash", "record_hash"};

// ---------------------------------------------------------------- Python-compatible JSON text
inline void put_codepoint_escape(std::string& o, unsigned cp) {
  char b[8];
  std::snprintf(b, sizeof b, "\\u%04x", cp);
  o += b;
}

// json.dumps string escaping: ensure_ascii=False keeps UTF-8 as is (canonical_json);
// ensure_ascii=True writes \uXXXX (surrogate pairs above the BMP) like the reader's --json.
inline void put_string(std::string& o, const std::string& s, bool ascii) {
  o.push_back('"');
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (c < 0x20) {
      put_codepoint_escape(o, c);
    } else if (c < 0x80 || !ascii) {
      o.push_back(static_cast<char>(c));
    } else {  // decode one UTF-8 sequence
      unsigned cp = 0;
      int extra = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : c >= 0xC0 ? 1 : 0;
      cp = c & (0x3F >> extra);
      for (int k = 0; k < extra && i + 1 < s.size(); ++k) cp = (cp << 6) | (static_cast<unsigned char>(s[++i]) & 0x3F);
      if (cp >= 0x10000) {
        cp -= 0x10000;
        put_codepoint_escape(o, 0xD800 + (cp >> 10));
        put_codepoint_escape(o, 0xDC00 + (cp & 0x3FF));
      } else {
        put_codepoint_escape(o, cp);
      }
    }
  }
  o.push_back('"');
}

inline std::string py_float(double d) {
  char b[40];
  for (int prec = 1; prec <= 17; ++prec) {  // shortest repr that round-trips, like Python's repr
    std::snprintf(b, sizeof b, "%.*g", prec, d);
    if (std::strtod(b, nullptr) == d) break;
  }
  std::string s = b;
  if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
  return s;
}

inline void put_value(std::string& o, const Json& v, bool ascii) {
  switch (v.type()) {
    case Json::Type::Null: o += "null"; break;
    case Json::Type::Bool: o += v.as_bool() ? "true" : "false"; break;
    case Json::Type::Int: o += std::to_string(v.as_int()); break;
    case Json::Type::Double: o += py_float(v.as_double()); break;
    case Json::Type::String: put_string(o, v.as_string(), ascii); break;
    case Json::Type::Array: {
      o.push_back('[');
      bool first = true;
      for (auto& e : v.items()) {
        if (!first) o.push_back(',');
        first = false;
        put_value(o, e, ascii);
      }
      o.push_back(']');
      break;
    }
    case Json::Type::Object: {
      o.push_back('{');
      bool first = true;
      for (auto& kv : v.fields()) {
        if (!first) o.push_back(',');
        first = false;
        put_string(o, kv.first, ascii);
        o.push_back(':');
        put_value(o, kv.second, ascii);
      }
      o.push_back('}');
      break;
    }
  }
}

inline std::string canonical_json(const Json& rec, bool null_hash) {
  std::string o = "{";
  bool first = true;
  for (const char* f : kFields) {
    if (!first) o.push_back(',');
    first = false;
    put_string(o, f, false);
    o.push_back(':');
    if (null_hash && std::strcmp(f, "record_hash") == 0) o += "null";
    else put_value(o, rec[f], false);
  }
  return o + "}";
}

inline std::string hmac_hex(const std::string& secret, const std::string& msg) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  HMAC(EVP_sha256(), secret.data(), static_cast<int>(secret.size()), reinterpret_cast<const unsigned char*>(msg.data()),
       msg.size(), md, &len);
  static const char* hex = "0123456789abcdef";
  std::string out;
  for (unsigned i = 0; i < len; ++i) {
    out.push_back(hex[md[i] >> 4]);
    out.push_back(hex[md[i] & 15]);
  }
  return out;
}

}  // namespace audit
}  // namespace dfs
