// audit_reader — read, filter and verify the S3 gateway's audit log (C59; reference
// dfs/s3_server/src/bin/audit_reader.rs). Checked against the Python model tests/models/
// s3_audit.py::reader_main over the same segment store (seg-<hour_ms>.log with one
// "<key_ts>\t<canonical json>" line per record, seg-<h>.uidx / .ridx index lines
// "<user|bucket>\t<offset>\t<length>"), with the same flags and output:
//
//   audit_reader DB_PATH [-u USER] [-r RESOURCE] [-a ACTION] [-s STATUS] [--start ISO] [--end ISO]
//                [--json] [-l LIMIT] [--verify-chain SECRET]
//
// A user query, or a bucket query, reads only the index lines of each segment in the time
// range and seeks to the matching records; bytes past the last indexed record (a crash between
// the two appends, or a segment without indexes) are scanned and filtered by content.
// --verify-chain recomputes record_hash = HMAC-SHA256(secret, canonical JSON with
// record_hash = null) for every record in key order and checks each previous_hash link; the
// canonical JSON is rebuilt from the parsed record exactly as audit.py::canonical_json writes
// it (reference field order, compact separators, non-ASCII kept as UTF-8).
#include <dirent.h>
#include <openssl/hmac.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <functional>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "audit_json.h"
#include "json.h"

using dfs::Json;
using namespace dfs::audit;  // NOLINT: kFields, canonical_json, hmac_hex, put_value

namespace {

constexpr int64_t kHourMs = 3'600'000;
// ---------------------------------------------------------------- segment store
struct Rec {
  int64_t key = 0;
  Json j;
};

std::vector<std::pair<int64_t, std::string>> segments(const std::string& dir) {
  std::vector<std::pair<int64_t, std::string>> out;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    std::string n = e->d_name;
    if (n.size() > 8 && n.compare(0, 4, "seg-") == 0 && n.compare(n.size() - 4, 4, ".log") == 0) {
      const std::string num = n.substr(4, n.size() - 8);
      char* end = nullptr;
      long long v = std::strtoll(num.c_str(), &end, 10);
      if (end && *end == 0 && !num.empty()) out.emplace_back(v, dir + "/" + n);
    }
  }
  ::closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::optional<Rec> parse_line(std::string line) {
  while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
  const auto tab = line.find('\t');
  if (line.empty() || tab == std::string::npos) return std::nullopt;
  try {
    size_t used = 0;
    Rec r;
    r.key = std::stoll(line.substr(0, tab), &used);
    if (used != tab) return std::nullopt;
    r.j = Json::parse(line.substr(tab + 1));
    return r;
  } catch (const std::exception&) {
    return std::nullopt;
  }
}

bool in_range(int64_t ts, std::optional<int64_t> a, std::optional<int64_t> b) {
  return (!a || ts >= *a) && (!b || ts <= *b);
}

bool seg_skipped(int64_t seg, std::optional<int64_t> a, std::optional<int64_t> b, bool* stop) {
  if (b && seg > *b) {
    *stop = true;
    return true;
  }
  return a && seg + kHourMs <= *a;
}

std::string idx_key(const Json& v) {
  std::string s = v.is_string() ? v.as_string() : (v.is_null() ? "" : v.dump());
  for (auto& c : s)
    if (c == '\t' || c == '\n') c = ' ';
  return s;
}

std::string bucket_of(const std::string& resource) {
  std::vector<std::string> parts;
  std::string cur;
  for (char c : resource) {
    if (c == ':') {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  parts.push_back(cur);
  const std::string bid = parts.size() > 5 ? parts[5] : resource;
  return bid.substr(0, bid.find('/'));
}

// every record in the time range, in key order; `fn` returns false to stop
void scan(const std::string& dir, std::optional<int64_t> a, std::optional<int64_t> b,
          const std::function<bool(const Rec&)>& fn) {
  for (auto& [seg, path] : segments(dir)) {
    bool stop = false;
    if (seg_skipped(seg, a, b, &stop)) {
      if (stop) return;
      continue;
    }
    std::ifstream f(path, std::ios::binary);
    std::string line;
    while (std::getline(f, line)) {
      auto r = parse_line(line);
      if (r && in_range(r->key, a, b) && !fn(*r)) return;
    }
  }
}

// records whose user ("user") or bucket ("resource") is `want`, through the index files
void lookup(const std::string& dir, bool user, const std::string& value, std::optional<int64_t> a,
            std::optional<int64_t> b, const std::function<bool(const Rec&)>& fn) {
  std::string want = value;
  for (auto& c : want)
    if (c == '\t' || c == '\n') c = ' ';
  for (auto& [seg, path] : segments(dir)) {
    bool stop = false;
    if (seg_skipped(seg, a, b, &stop)) {
      if (stop) return;
      continue;
    }
    std::vector<std::pair<uint64_t, uint64_t>> refs;
    uint64_t covered = 0;
    std::ifstream idx(dir + "/seg-" + std::to_string(seg) + (user ? ".uidx" : ".ridx"));
    std::string line;
    while (std::getline(idx, line)) {
      const auto t1 = line.find('\t'), t2 = t1 == std::string::npos ? t1 : line.find('\t', t1 + 1);
      if (t2 == std::string::npos || line.find('\t', t2 + 1) != std::string::npos) continue;  // torn line
      try {
        const uint64_t off = std::stoull(line.substr(t1 + 1, t2 - t1 - 1)), ln = std::stoull(line.substr(t2 + 1));
        covered = std::max(covered, off + ln);
        if (line.compare(0, t1, want) == 0 && t1 == want.size()) refs.emplace_back(off, ln);
      } catch (const std::exception&) {
      }
    }
    std::ifstream f(path, std::ios::binary);
    std::string buf;
    for (auto& [off, ln] : refs) {
      buf.assign(ln, '\0');
      f.clear();
      f.seekg(static_cast<std::streamoff>(off));
      f.read(&buf[0], static_cast<std::streamsize>(ln));
      auto r = parse_line(buf.substr(0, static_cast<size_t>(f.gcount())));
      if (r && in_range(r->key, a, b) && !fn(*r)) return;
    }
    f.clear();
    f.seekg(static_cast<std::streamoff>(covered));
    while (std::getline(f, line)) {  // unindexed tail: filter by content
      auto r = parse_line(line);
      if (!r || !in_range(r->key, a, b)) continue;
      const std::string field = user ? idx_key(r->j["user_id"]) : idx_key(Json(bucket_of(r->j["resource"].str())));
      if (field == want && !fn(*r)) return;
    }
  }
}

// datetime.fromisoformat(s.replace("Z", "+00:00")).timestamp() * 1000 (naive = local time)
std::optional<int64_t> parse_time(std::string s) {
  for (size_t p; (p = s.find('Z')) != std::string::npos;) s.replace(p, 1, "+00:00");
  std::tm tm{};
  int y = 0, mo = 0, d = 0, h = 0, mi = 0;
  double sec = 0;
  int n = 0;
  if (std::sscanf(s.c_str(), "%4d-%2d-%2d%n", &y, &mo, &d, &n) != 3) return std::nullopt;
  size_t pos = static_cast<size_t>(n);
  if (pos < s.size() && (s[pos] == 'T' || s[pos] == ' ')) {
    int m2 = 0;
    if (std::sscanf(s.c_str() + pos + 1, "%2d:%2d%n", &h, &mi, &m2) != 2) return std::nullopt;
    pos += 1 + static_cast<size_t>(m2);
    if (pos < s.size() && s[pos] == ':') {
      char* end = nullptr;
      sec = std::strtod(s.c_str() + pos + 1, &end);
      pos = static_cast<size_t>(end - s.c_str());
    }
  }
  std::optional<int> tz_min;
  if (pos < s.size() && (s[pos] == '+' || s[pos] == '-')) {
    int th = 0, tmi = 0;
    if (std::sscanf(s.c_str() + pos + 1, "%2d:%2d", &th, &tmi) < 1) return std::nullopt;
    tz_min = (s[pos] == '-' ? -1 : 1) * (th * 60 + tmi);
  } else if (pos != s.size()) {
    return std::nullopt;
  }
  tm.tm_year = y - 1900;
  tm.tm_mon = mo - 1;
  tm.tm_mday = d;
  tm.tm_hour = h;
  tm.tm_min = mi;
  tm.tm_sec = 0;
  tm.tm_isdst = -1;
  time_t t = tz_min ? ::timegm(&tm) - static_cast<time_t>(*tz_min) * 60 : std::mktime(&tm);
  return static_cast<int64_t>(t) * 1000 + static_cast<int64_t>(sec * 1000.0);
}

std::string field_text(const Json& rec, const char* k) {  // audit.py::_txt: "" for null or missing
  const Json* v = rec.find(k);
  if (!v) return "";
  switch (v->type()) {
    case Json::Type::Null: return "";
    case Json::Type::Bool: return v->as_bool() ? "True" : "False";
    case Json::Type::Int: return std::to_string(v->as_int());
    case Json::Type::Double: return py_float(v->as_double());
    case Json::Type::String: return v->as_string();
    default: {
      std::string o;
      put_value(o, *v, false);
      return o;
    }
  }
}

std::string pad(const std::string& s, size_t w) {  // <w on code points, like Python
  size_t cps = 0;
  for (unsigned char c : s) cps += (c & 0xC0) != 0x80;
  return cps >= w ? s : s + std::string(w - cps, ' ');
}

int usage() {
  std::fprintf(stderr,
               "usage: audit_reader DB_PATH [-u USER] [-r RESOURCE] [-a ACTION] [-s STATUS] [--start ISO] [--end ISO] "
               "[--json] [-l LIMIT] [--verify-chain SECRET]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::string db, user, resource, action, secret;
  std::optional<int64_t> status, start, end;
  bool as_json = false, verify = false;
  long limit = 100;
  for (int i = 1; i < argc; ++i) {
    const std::string s = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + s);
      return argv[++i];
    };
    try {
      if (s == "-u" || s == "--user") user = val();
      else if (s == "-r" || s == "--resource") resource = val();
      else if (s == "-a" || s == "--action") action = val();
      else if (s == "-s" || s == "--status") status = std::stoll(val());
      else if (s == "--start" || s == "--end") {
        auto t = parse_time(val());
        if (!t) throw std::runtime_error("invalid time for " + s);
        (s == "--start" ? start : end) = t;
      } else if (s == "--json") as_json = true;
      else if (s == "-l" || s == "--limit") limit = std::stol(val());
      else if (s == "--verify-chain") {
        secret = val();
        verify = true;
      } else if (s == "-h" || s == "--help") {
        usage();
        return 0;
      } else if (!s.empty() && s[0] == '-') {
        std::fprintf(stderr, "audit_reader: unknown option %s\n", s.c_str());
        return usage();
      } else if (db.empty()) {
        db = s;
      } else {
        return usage();
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "audit_reader: %s\n", e.what());
      return usage();
    }
  }
  if (db.empty()) return usage();
  while (db.size() > 1 && db.back() == '/') db.pop_back();

  if (verify) {
    std::vector<std::string> errors;
    Json prev;  // null
    size_t n = 0;
    scan(db, std::nullopt, std::nullopt, [&](const Rec& r) {
      ++n;
      const std::string who = "record " + field_text(r.j, "request_id") + " @ " + std::to_string(r.key);
      if (r.j["previous_hash"] != prev) errors.push_back(who + ": previous_hash does not link");
      if (!(r.j["record_hash"].is_string() && hmac_hex(secret, canonical_json(r.j, true)) == r.j["record_hash"].str()))
        errors.push_back(who + ": record_hash mismatch");
      prev = r.j["record_hash"];
      return true;
    });
    for (auto& e : errors) std::printf("%s\n", e.c_str());
    if (errors.empty()) std::printf("verified %zu records: OK\n", n);
    else std::printf("verified %zu records: %zu errors\n", n, errors.size());
    return errors.empty() ? 0 : 1;
  }

  long count = 0;
  if (!as_json) std::printf("%-32s %-20s %-22s %-6s RESOURCE\n", "TIMESTAMP", "USER", "ACTION", "STATUS");
  auto emit = [&](const Rec& r) {
    const Json& j = r.j;
    if (!user.empty() && !(j["user_id"].is_string() && j["user_id"].as_string() == user)) return true;
    if (!resource.empty() && bucket_of(j["resource"].str()) != resource && j["resource"].str() != resource) return true;
    if (!action.empty() && !(j["action"].is_string() && j["action"].as_string() == action)) return true;
    if (status && !(j["status_code"].is_int() && j["status_code"].as_int() == *status)) return true;
    if (as_json) {
      std::string o;
      put_value(o, j, true);
      std::printf("%s\n", o.c_str());
    } else {
      std::printf("%s %s %s %s %s\n", pad(field_text(j, "timestamp"), 32).c_str(), pad(field_text(j, "user_id"), 20).c_str(),
                  pad(field_text(j, "action"), 22).c_str(), pad(field_text(j, "status_code"), 6).c_str(),
                  field_text(j, "resource").c_str());
    }
    return ++count < limit;
  };
  if (!user.empty()) lookup(db, true, user, start, end, emit);
  else if (!resource.empty() && resource.find(':') == std::string::npos && resource.find('/') == std::string::npos)
    lookup(db, false, resource, start, end, emit);
  else scan(db, start, end, emit);
  if (!as_json && count == 0) std::printf("no matching records\n");
  return 0;
}
