// JSON serialisation (see json.h). UTF-8 passes through unescaped, which Python's json
// module and serde_json both read back unchanged.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "json.h"

namespace dfs {

void json_escape(const std::string& s, std::string& out) {
  out.push_back('"');
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
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

void Json::dump_to(std::string& out) const {
  switch (t_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: {
      if (std::isnan(d_)) {
        out += "NaN";
      } else if (std::isinf(d_)) {
        out += d_ > 0 ? "Infinity" : "-Infinity";
      } else {
        char buf[32];
        std::snprintf(buf, sizeof buf, "%.17g", d_);
        out += buf;
        if (!std::strpbrk(buf, ".eEn")) out += ".0";
      }
      break;
    }
    case Type::String: json_escape(s_, out); break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        v.dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (auto& kv : *o_) {
        if (!first) out.push_back(',');
        first = false;
        json_escape(kv.first, out);
        out.push_back(':');
        kv.second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out);
  return out;
}

}  // namespace dfs
