// otlp_columnizer.cc -- see otlp_columnizer.h.
#include "otlp_columnizer.h"

#include <sys/mman.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <string_view>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <chrono>
#include <mutex>
#include <thread>

namespace otlpcol {
namespace {

// ---------------------------------------------------------------- xxHash64
constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t *p) {
  uint64_t v;
  std::memcpy(&v, p, 8);  // little-endian host (x86-64)
  return v;
}
inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t round1(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
inline uint64_t merge1(uint64_t acc, uint64_t v) { return (acc ^ round1(0, v)) * P1 + P4; }

// ---------------------------------------------------------------- protobuf
struct PB {
  const uint8_t *p, *end;
  bool ok = true;
  PB(const uint8_t *a, const uint8_t *b) : p(a), end(b) {}
  void fail() { ok = false; p = end; }
  uint64_t varint() {
    if (p < end && *p < 0x80) return *p++;  // one byte: tags, kinds, short lengths
    uint64_t x = 0;
    for (int s = 0; s < 64 && p < end; s += 7) {
      const uint8_t b = *p++;
      x |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return x;
    }
    fail();
    return 0;
  }
  uint64_t fixed64() {
    if (end - p < 8) return fail(), 0;
    const uint64_t v = rd64(p);
    p += 8;
    return v;
  }
  double dbl() {
    const uint64_t u = fixed64();
    double d;
    std::memcpy(&d, &u, 8);
    return d;
  }
  PB sub() {
    const uint64_t n = varint();
    if (!ok || n > (uint64_t)(end - p)) {
      fail();
      return PB(end, end);
    }
    PB s(p, p + n);
    p += n;
    return s;
  }
  std::string_view str() {
    PB s = sub();
    return std::string_view(reinterpret_cast<const char *>(s.p), (size_t)(s.end - s.p));
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: if (end - p < 8) fail(); else p += 8; break;
      case 2: sub(); break;
      case 5: if (end - p < 4) fail(); else p += 4; break;
      default: fail();
    }
  }
  // next field; false at the end or on error (check ok)
  bool next(uint32_t &f, int &wt) {
    if (p >= end) return false;
    const uint64_t t = varint();
    if (!ok) return false;
    f = (uint32_t)(t >> 3);
    wt = (int)(t & 7);
    if (f == 0) return fail(), false;
    return true;
  }
};

// ---------------------------------------------------------------- strings
bool valid_utf8(std::string_view s) {
  const auto *p = reinterpret_cast<const uint8_t *>(s.data()), *e = p + s.size();
  while (p < e) {
    const uint8_t c = *p;
    if (c < 0x80) { ++p; continue; }
    int n;
    uint32_t cp;
    if ((c & 0xE0) == 0xC0) n = 1, cp = c & 0x1F;
    else if ((c & 0xF0) == 0xE0) n = 2, cp = c & 0x0F;
    else if ((c & 0xF8) == 0xF0) n = 3, cp = c & 0x07;
    else return false;
    if (e - p <= n) return false;
    for (int i = 1; i <= n; ++i) {
      if ((p[i] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (p[i] & 0x3F);
    }
    if ((n == 1 && cp < 0x80) || (n == 2 && cp < 0x800) || (n == 3 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    p += n + 1;
  }
  return true;
}

std::vector<uint32_t> code_points(std::string_view s) {  // s is valid UTF-8
  std::vector<uint32_t> out;
  const auto *p = reinterpret_cast<const uint8_t *>(s.data()), *e = p + s.size();
  while (p < e) {
    const uint8_t c = *p;
    int n = c < 0x80 ? 0 : (c & 0xE0) == 0xC0 ? 1 : (c & 0xF0) == 0xE0 ? 2 : 3;
    uint32_t cp = n == 0 ? c : n == 1 ? (c & 0x1F) : n == 2 ? (c & 0x0F) : (c & 0x07);
    for (int i = 1; i <= n; ++i) cp = (cp << 6) | (p[i] & 0x3F);
    out.push_back(cp);
    p += n + 1;
  }
  return out;
}

const char *kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
std::string base64(std::string_view b) {
  std::string o;
  o.reserve((b.size() + 2) / 3 * 4);
  size_t i = 0;
  const auto *u = reinterpret_cast<const uint8_t *>(b.data());
  for (; i + 3 <= b.size(); i += 3) {
    const uint32_t v = (u[i] << 16) | (u[i + 1] << 8) | u[i + 2];
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += kB64[v & 63];
  }
  if (b.size() - i == 1) {
    const uint32_t v = u[i] << 16;
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += "==";
  } else if (b.size() - i == 2) {
    const uint32_t v = (u[i] << 16) | (u[i + 1] << 8);
    o += kB64[v >> 18]; o += kB64[(v >> 12) & 63]; o += kB64[(v >> 6) & 63]; o += '=';
  }
  return o;
}

// JSON.stringify of a (valid UTF-8) string
void json_string(std::string &o, std::string_view s) {
  static const char *hex = "0123456789abcdef";
  o += '"';
  for (const char ch : s) {
    const uint8_t c = (uint8_t)ch;
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          o += "\\u00";
          o += hex[c >> 4];
          o += hex[c & 15];
        } else {
          o += ch;
        }
    }
  }
  o += '"';
}

// shortest round-trip digits and decimal exponent: v = 0.d1d2... * 10^n (JS's n)
void shortest(double v, std::string &digits, int &n) {
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string_view s(buf, (size_t)(r.ptr - buf));  // d[.ddd]e±xx
  const size_t epos = s.find('e');
  digits.clear();
  for (size_t i = 0; i < epos; ++i)
    if (s[i] != '.') digits += s[i];
  int e = 0;
  std::from_chars(s.data() + epos + 1 + (s[epos + 1] == '+'), s.data() + s.size(), e);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  n = e + 1;
}

// JavaScript Number.prototype.toString() for finite v
std::string js_number(double v) {
  if (v == 0) return "0";
  std::string sign = std::signbit(v) ? "-" : "";
  std::string d;
  int n;
  shortest(std::fabs(v), d, n);
  const int k = (int)d.size();
  if (k <= n && n <= 21) return sign + d + std::string(n - k, '0');
  if (0 < n && n <= 21) return sign + d.substr(0, n) + "." + d.substr(n);
  if (-6 < n && n <= 0) return sign + "0." + std::string(-n, '0') + d;
  const int e = n - 1;
  std::string o = sign + d.substr(0, 1);
  if (k > 1) o += "." + d.substr(1);
  return o + "e" + (e >= 0 ? "+" : "-") + std::to_string(std::abs(e));
}

// ---------------------------------------------------------------- AnyValue
enum VType { kEmpty, kStr, kBool, kInt, kDouble, kBytes, kArray, kKvlist };
const char *kTypeTag[] = {"NoneType", "str", "bool", "int", "float", "bytes", "list", "dict"};

struct Any {
  VType type = kEmpty;
  std::string_view s;  // kStr / kBytes
  bool b = false;
  int64_t i = 0;
  double d = 0;
  PB body{nullptr, nullptr};  // kArray / kKvlist
};

Any parse_any(PB pb) {
  Any a;  // last field wins, like otlp.js decodeAnyValue
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) a = Any{}, a.type = kStr, a.s = pb.str();
    else if (f == 2 && wt == 0) a = Any{}, a.type = kBool, a.b = pb.varint() != 0;
    else if (f == 3 && wt == 0) a = Any{}, a.type = kInt, a.i = (int64_t)pb.varint();
    else if (f == 4 && wt == 1) a = Any{}, a.type = kDouble, a.d = pb.dbl();
    else if (f == 5 && wt == 2) a = Any{}, a.type = kArray, a.body = pb.sub();
    else if (f == 6 && wt == 2) a = Any{}, a.type = kKvlist, a.body = pb.sub();
    else if (f == 7 && wt == 2) a = Any{}, a.type = kBytes, a.s = pb.str();
    else pb.skip(wt);
  }
  if (!pb.ok) a.type = kEmpty, a.body = PB(nullptr, nullptr), a.s = {}, a.i = 0;
  return a;
}

// Nesting limit for array / kvlist attribute values (Go's protobuf decoder
// also bounds recursion): a deeper value makes the request malformed instead
// of recursing on the native stack.
constexpr int kMaxAnyDepth = 100;

// Structure of an AnyValue body (nested arrays / kvlists included) down to
// kMaxAnyDepth levels: false when malformed or nested deeper.
bool valid_any_body(PB pb, int depth);
bool valid_nested(PB pb, bool kvlist, int depth) {
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) {
      PB item = pb.sub();
      if (!kvlist) {
        if (!valid_any_body(item, depth + 1)) return false;
      } else {
        uint32_t g;
        int wt2;
        while (item.next(g, wt2)) {
          if (g == 2 && wt2 == 2) {
            if (!valid_any_body(item.sub(), depth + 1)) return false;
          } else {
            item.skip(wt2);
          }
        }
        if (!item.ok) return false;
      }
    } else {
      pb.skip(wt);
    }
  }
  return pb.ok;
}
bool valid_any_body(PB pb, int depth) {
  if (depth > kMaxAnyDepth) return false;
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if ((f == 5 || f == 6) && wt == 2) {
      if (!valid_nested(pb.sub(), f == 6, depth)) return false;
    } else {
      pb.skip(wt);
    }
  }
  return pb.ok;
}

// parse_any and valid_any_body(pb, 0) in one walk over the body: the value
// (last field wins) and, in ok, whether the body is well formed (every array
// or kvlist field in it checked, as valid_any_body does)
Any parse_any_valid(PB pb, bool &ok) {
  Any a;
  ok = true;
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) a = Any{}, a.type = kStr, a.s = pb.str();
    else if (f == 2 && wt == 0) a = Any{}, a.type = kBool, a.b = pb.varint() != 0;
    else if (f == 3 && wt == 0) a = Any{}, a.type = kInt, a.i = (int64_t)pb.varint();
    else if (f == 4 && wt == 1) a = Any{}, a.type = kDouble, a.d = pb.dbl();
    else if ((f == 5 || f == 6) && wt == 2) {
      a = Any{}, a.type = f == 5 ? kArray : kKvlist, a.body = pb.sub();
      if (ok && !valid_nested(a.body, f == 6, 0)) ok = false;
    } else if (f == 7 && wt == 2) a = Any{}, a.type = kBytes, a.s = pb.str();
    else pb.skip(wt);
  }
  if (!pb.ok) a.type = kEmpty, a.body = PB(nullptr, nullptr), a.s = {}, a.i = 0, ok = false;
  return a;
}

// KeyValue -> (key, value); false on malformed input, a malformed or too
// deeply nested value included (the request is then rejected, as the Go
// collector's unmarshal and otlp.js reject it)
bool parse_kv(PB pb, std::string_view &key, Any &val) {
  key = {};
  val = Any{};
  bool vok = true;
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) {
      key = pb.str();
    } else if (f == 2 && wt == 2) {
      val = parse_any_valid(pb.sub(), vok);
    } else {
      pb.skip(wt);
    }
  }
  return pb.ok && vok;
}
enum class Keyable { kYes, kNotNative, kTooDeep };

Keyable raw_json(std::string &o, const Any &a, int depth);

Keyable raw_json_array(std::string &o, PB pb, int depth) {
  o += '[';
  bool first = true;
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) {
      if (!first) o += ',';
      first = false;
      const Keyable k = raw_json(o, parse_any(pb.sub()), depth + 1);
      if (k != Keyable::kYes) return k;
    } else {
      pb.skip(wt);
    }
  }
  o += ']';
  return pb.ok ? Keyable::kYes : Keyable::kNotNative;
}

Keyable raw_json_kvlist(std::string &o, PB pb, int depth) {
  o += '{';
  bool first = true;
  uint32_t f;
  int wt;
  while (pb.next(f, wt)) {
    if (f == 1 && wt == 2) {
      std::string_view k;
      Any v;
      if (!parse_kv(pb.sub(), k, v) || !valid_utf8(k)) return Keyable::kNotNative;
      if (!first) o += ',';
      first = false;
      json_string(o, k);
      o += ':';
      const Keyable kk = raw_json(o, v, depth + 1);
      if (kk != Keyable::kYes) return kk;
    } else {
      pb.skip(wt);
    }
  }
  o += '}';
  return pb.ok ? Keyable::kYes : Keyable::kNotNative;
}

// keys.js rawJson
Keyable raw_json(std::string &o, const Any &a, int depth) {
  switch (a.type) {
    case kStr:
      if (!valid_utf8(a.s)) return Keyable::kNotNative;
      json_string(o, a.s);
      return Keyable::kYes;
    case kBool: o += a.b ? "true" : "false"; return Keyable::kYes;
    case kInt: o += std::to_string(a.i); return Keyable::kYes;
    case kDouble:
      if (std::isfinite(a.d)) o += js_number(a.d);
      else json_string(o, format_float(a.d));
      return Keyable::kYes;
    case kBytes: json_string(o, base64(a.s)); return Keyable::kYes;
    case kArray:
      return depth >= kMaxAnyDepth ? Keyable::kTooDeep : raw_json_array(o, a.body, depth);
    case kKvlist:
      return depth >= kMaxAnyDepth ? Keyable::kTooDeep : raw_json_kvlist(o, a.body, depth);
    default: o += "null"; return Keyable::kYes;
  }
}

// keys.js asString; kNotNative when the value cannot be keyed natively (the
// JavaScript columnizer takes the request), kTooDeep for a malformed request
Keyable as_string(const Any &a, std::string &o) {
  o.clear();
  switch (a.type) {
    case kStr:
      if (!valid_utf8(a.s)) return Keyable::kNotNative;
      o.assign(a.s);
      return Keyable::kYes;
    case kBool: o = a.b ? "true" : "false"; return Keyable::kYes;
    case kInt: o = std::to_string(a.i); return Keyable::kYes;
    case kDouble: o = format_float(a.d); return Keyable::kYes;
    case kBytes: o = base64(a.s); return Keyable::kYes;
    case kArray: case kKvlist: return raw_json(o, a, 1);
    default: return Keyable::kYes;
  }
}

const char *kKindStr[] = {"SPAN_KIND_UNSPECIFIED", "SPAN_KIND_INTERNAL", "SPAN_KIND_SERVER",
                          "SPAN_KIND_CLIENT", "SPAN_KIND_PRODUCER", "SPAN_KIND_CONSUMER"};
const char *kStatusStr[] = {"STATUS_CODE_UNSET", "STATUS_CODE_OK", "STATUS_CODE_ERROR"};

bool glob_match(const std::vector<uint32_t> &pat, const std::vector<uint32_t> &s) {
  size_t p = 0, i = 0, star = std::string::npos, mark = 0;
  while (i < s.size()) {
    if (p < pat.size() && (pat[p] == '?' || (pat[p] != '*' && pat[p] == s[i]))) {
      ++p, ++i;
    } else if (p < pat.size() && pat[p] == '*') {
      star = p++;
      mark = i;
    } else if (star != std::string::npos) {
      p = star + 1;
      i = ++mark;
    } else {
      return false;
    }
  }
  while (p < pat.size() && pat[p] == '*') ++p;
  return p == pat.size();
}

struct Attr {
  std::string_view key;
  Any val;
};

// attrMap semantics: one entry per key, the last value wins
void dedupe_last(std::vector<Attr> &v) {
  std::vector<Attr> out;
  out.reserve(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    bool later = false;
    for (size_t j = i + 1; j < v.size() && !later; ++j) later = v[j].key == v[i].key;
    if (!later) out.push_back(v[i]);
  }
  v.swap(out);
}

const Any *find_attr(const std::vector<Attr> &v, std::string_view k) {
  for (auto it = v.rbegin(); it != v.rend(); ++it)
    if (it->key == k) return &it->val;
  return nullptr;
}



}  // namespace

uint64_t xxh64(const void *data, size_t len, uint64_t seed) {
  const uint8_t *p = static_cast<const uint8_t *>(data), *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t *limit = end - 32;
    do {
      v1 = round1(v1, rd64(p));
      v2 = round1(v2, rd64(p + 8));
      v3 = round1(v3, rd64(p + 16));
      v4 = round1(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge1(h, v1);
    h = merge1(h, v2);
    h = merge1(h, v3);
    h = merge1(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  for (; p + 8 <= end; p += 8) h = rotl(h ^ round1(0, rd64(p)), 27) * P1 + P4;
  if (p + 4 <= end) {
    h = rotl(h ^ ((uint64_t)rd32(p) * P1), 23) * P2 + P3;
    p += 4;
  }
  for (; p < end; ++p) h = rotl(h ^ ((uint64_t)*p * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

std::string format_float(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return std::signbit(v) ? "-0" : "0";
  std::string d;
  int n;
  shortest(std::fabs(v), d, n);
  const std::string sign = v < 0 ? "-" : "";
  const int k = (int)d.size();
  if (n >= k) return sign + d + std::string(n - k, '0');
  if (n > 0) return sign + d.substr(0, n) + "." + d.substr(n);
  return sign + "0." + std::string(-n, '0') + d;
}

void Rule::prepare() {
  cps = code_points(pattern);
  prefix.clear();
  for (char c : pattern) {
    if (c == '*' || c == '?') break;
    prefix += c;
  }
}

std::string apply_rules(const std::vector<Rule> &rules, std::string name) {
  for (const Rule &r : rules) {  // kGlob rules must have been prepare()d
    if (r.kind == Rule::kStripQuery) {
      // Go regexp `\?.*`, ReplaceAllString(.., ""): `.` stops at '\n'
      std::string o;
      o.reserve(name.size());
      for (size_t i = 0; i < name.size();) {
        if (name[i] == '?') {
          while (i < name.size() && name[i] != '\n') ++i;
        } else {
          o += name[i++];
        }
      }
      name.swap(o);
    } else if (name.compare(0, r.prefix.size(), r.prefix) == 0 &&
               glob_match(r.cps, code_points(name))) {
      name = r.replacement;
    }
  }
  return name;
}

uint32_t Columnizer::service_id(const std::string &name, bool *is_new) {
  auto it = services_.find(name);
  if (it != services_.end()) {
    if (is_new) *is_new = false;
    return it->second;
  }
  const uint32_t id = (uint32_t)std::min<size_t>(services_.size(), 0xFFFE);  // 0xFFFF: event records
  services_.emplace(name, id);
  if (is_new) *is_new = true;
  return id;
}

// ---------------------------------------------------------------- columns, caches, threads
namespace {
HostAllocFn g_host_alloc = nullptr;
HostFreeFn g_host_free = nullptr;
constexpr size_t kColHdr = 64;  // block header: the block's kind (1 = page-locked), keeps 64-B alignment
}  // namespace

void set_host_allocator(HostAllocFn a, HostFreeFn f) {
  g_host_alloc = a;
  g_host_free = f;
}

void *col_alloc(size_t bytes, bool pinned) {
  unsigned char *raw = nullptr;
  uint64_t kind = 0;
  if (pinned && g_host_alloc) {
    raw = static_cast<unsigned char *>(g_host_alloc(bytes + kColHdr));
    kind = raw ? 1 : 0;
  }
  if (!raw) raw = static_cast<unsigned char *>(::operator new(bytes + kColHdr, std::align_val_t(kColHdr)));
  *reinterpret_cast<uint64_t *>(raw) = kind;
  return raw + kColHdr;
}

void col_free(void *p) {
  if (!p) return;
  unsigned char *raw = static_cast<unsigned char *>(p) - kColHdr;
  if (*reinterpret_cast<uint64_t *>(raw) == 1 && g_host_free) g_host_free(raw);
  else ::operator delete(raw, std::align_val_t(kColHdr));
}

void Cols::reserve(size_t cap) {
  if (cap <= key.size()) return;
  const size_t c = std::max<size_t>({cap, 2 * key.size(), 4096});
  key.resize(c), start.resize(c), end.resize(c), w0.resize(c), w1.resize(c), meta.resize(c);
}

// The cache's own hash (any good mix will do; names are compared on a hit):
// 8-byte words of the name, the last one overlapping, through a multiply-xorshift.
uint64_t SigCache::hash(uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind, int32_t code) {
  constexpr uint64_t K = 0x9E3779B97F4A7C15ULL;
  uint64_t h = rhash ^ ((uint64_t)svc << 40) ^ ((uint64_t)(uint32_t)kind << 8) ^ (uint32_t)code ^
               ((uint64_t)name.size() << 56);
  auto mix = [&](uint64_t v) {
    h = (h ^ v) * K;
    h ^= h >> 29;
  };
  const auto *q = reinterpret_cast<const uint8_t *>(name.data());
  const size_t n = name.size();
  if (n >= 8) {
    size_t i = 0;
    for (; i + 8 < n; i += 8) mix(rd64(q + i));
    mix(rd64(q + n - 8));
  } else if (n >= 4) {
    mix(((uint64_t)rd32(q) << 32) | rd32(q + n - 4));
  } else if (n) {
    mix(((uint64_t)q[0] << 16) | ((uint64_t)q[n / 2] << 8) | q[n - 1]);
  }
  h = (h ^ (h >> 32)) * K;
  return (h ^ (h >> 29)) | 1;  // 0 never names a used slot
}

template <typename T>
void BigArray<T>::assign_zero(size_t n) {
  std::free(p_);
  p_ = nullptr, n_ = 0;
  if (!n) return;
  constexpr size_t kHuge = (size_t)2 << 20;
  size_t bytes = n * sizeof(T);
  void *q;
  if (bytes >= kHuge) {
    bytes = (bytes + kHuge - 1) / kHuge * kHuge;
    q = std::aligned_alloc(kHuge, bytes);
    if (q) madvise(q, bytes, MADV_HUGEPAGE);  // (advice only: a refusal changes nothing)
  } else {
    bytes = (bytes + 63) / 64 * 64;
    q = std::aligned_alloc(64, bytes);
  }
  if (!q) throw std::bad_alloc();
  std::memset(q, 0, bytes);
  p_ = static_cast<T *>(q), n_ = n;
}

const SigCache::Rec *SigCache::find(uint64_t h, uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind,
                                    int32_t code) const {
  if (recs_.empty()) return nullptr;
  const size_t mask = recs_.size() - 1;
  const uint32_t n = (uint32_t)name.size();
  for (size_t i = h & mask;; i = (i + 1) & mask) {
    const Rec &r = recs_[i];
    if (!r.h) return nullptr;
    if (r.h != h) continue;
    // a short name is compared in the record, a longer one in the arena
    // (which holds every name whole: one compare either way)
    if (r.rhash == rhash && r.svc == svc && r.kind == kind && r.code == code && r.name_len == n &&
        std::memcmp(n <= kInline ? r.name : names_.data() + r.name_off, name.data(), n) == 0)
      return &r;
  }
}

void SigCache::insert(uint64_t h, uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind,
                      int32_t code, uint64_t sid, const std::string &key) {
  if (!cacheable(kind, code)) return;
  if (2 * (entries_.size() + 1) > recs_.size()) {  // load <= 1/2: rebuild the records
    BigArray<Rec> old;
    old.swap(recs_);
    recs_.assign_zero(old.empty() ? 256 : old.size() * 2);
    const size_t mask = recs_.size() - 1;
    for (const Rec &o : old) {
      if (!o.h) continue;
      size_t i = o.h & mask;
      while (recs_[i].h) i = (i + 1) & mask;
      recs_[i] = o;
    }
  }
  const size_t mask = recs_.size() - 1;
  size_t i = h & mask;
  while (recs_[i].h) i = (i + 1) & mask;
  Rec &r = recs_[i];
  r.h = h;  // (never 0: hash() sets bit 0)
  r.sid = sid, r.rhash = rhash, r.svc = svc, r.kind = (int16_t)kind, r.code = (int16_t)code;
  r.name_len = (uint32_t)name.size(), r.name_off = (uint32_t)names_.size(), r.idx = (uint32_t)entries_.size();
  std::memcpy(r.name, name.data(), name.size() < kInline ? name.size() : kInline);
  fresh_.push_back((uint32_t)entries_.size());
  Entry e;
  e.h = h, e.rhash = rhash, e.sid = sid, e.svc = svc, e.kind = kind, e.code = code;
  e.name_off = (uint32_t)names_.size(), e.name_len = (uint32_t)name.size();
  names_.append(name);
  e.key = key;
  entries_.push_back(std::move(e));
}

namespace {
// a span of the batched path (run): what a signature-cache hit needs
struct FastSpan {
  const uint8_t *at;     // the span's field in its ScopeSpans (the full path restarts there on a miss)
  const uint8_t *name;   // the raw span name (no dimensions) or -- with dimensions -- noff into the arena
  uint32_t nlen = 0, noff = 0;
  int32_t kind = 0, code = 0;
  uint64_t sig = 0, st = 0, en = 0, w0 = 0, w1 = 0;
  bool slow = false;
};
constexpr size_t kBatch = 16;
constexpr size_t kBatchAbove = 1u << 16;  // own-cache signatures past which run() batches

// One ScopeSpans of run()'s batched path (neither exemplars nor events, and
// lookups that miss the CPU caches): spans are parsed kBatch at a time, each
// one's signature-cache records prefetched as soon as its hash is known, then
// resolved in order, so a batch's memory accesses overlap instead of
// following each other.  A span it cannot resolve (unknown signature, a
// dimension value that is not a string, anything malformed) goes back to
// run()'s full path, which keys it, reports it or fails as always.
struct BatchScope {
  std::vector<FastSpan> &pend;
  std::string &arena;
  std::vector<std::string_view> &dv;
  std::vector<uint8_t> &dt;
  bool own;  // probe the thread's own cache
  const std::vector<Dim> &dims;
  const std::vector<Attr> &rattrs;
  uint64_t rhash;
  uint32_t svc_id;
  const SigCache &cache;
  const SigCache *l2;
  Cols &out;
  uint64_t &spans, &own_misses;
};
// Emits the hits up to the next span the full path must take (true, with ss
// back at that span's field) or to the scope's end (false).  Out of line:
// run()'s plain loop stays as compact as it was without this path.
__attribute__((noinline)) bool batch_hits(BatchScope &b, PB &ss) {
  auto &pend = b.pend;
  std::string &arena = b.arena;
  const size_t nd = b.dims.size();
  for (;;) {
    {  // parse the next batch
      pend.clear();
      arena.clear();
      uint32_t h;
      int wt3;
      const uint8_t *at = ss.p;
      while (pend.size() < kBatch && ss.next(h, wt3)) {
        if (h != 2 || wt3 != 2) {
          ss.skip(wt3);
          at = ss.p;
          continue;
        }
        PB sp = ss.sub();
        pend.emplace_back();
        FastSpan &p = pend.back();
        p.at = at;
        at = ss.p;
        const uint8_t *tid = nullptr;
        size_t tid_len = 0;
        std::string_view name;
        int32_t kind = 0, code = 0;
        uint64_t st = 0, en = 0;
        // (per dimension: its last string value among the span attributes;
        // type 2 = a value of another type, which the full path keys)
        auto &dv = b.dv;
        auto &dt = b.dt;
        dv.assign(nd, std::string_view());
        dt.assign(nd, 0);
        bool slow = false;
        uint32_t k;
        int wt4;
        while (sp.next(k, wt4)) {
          if (k == 1 && wt4 == 2) {
            const std::string_view t = sp.str();
            tid = reinterpret_cast<const uint8_t *>(t.data());
            tid_len = t.size();
          } else if (k == 5 && wt4 == 2) {
            name = sp.str();
          } else if (k == 6 && wt4 == 0) {
            kind = (int32_t)(uint32_t)sp.varint();
          } else if (k == 7 && wt4 == 1) {
            st = sp.fixed64();
          } else if (k == 8 && wt4 == 1) {
            en = sp.fixed64();
          } else if (k == 9 && wt4 == 2 && nd) {
            std::string_view key;
            Any v;
            if (!parse_kv(sp.sub(), key, v)) {
              slow = true;
              continue;
            }
            for (size_t d = 0; d < nd; ++d)
              if (b.dims[d].name == key) dt[d] = v.type == kStr ? 1 : 2, dv[d] = v.s;
          } else if (k == 15 && wt4 == 2) {
            PB stt = sp.sub();
            uint32_t m;
            int wt5;
            code = 0;  // a later Status message replaces an earlier one
            while (stt.next(m, wt5)) {
              if (m == 3 && wt5 == 0) code = (int32_t)(uint32_t)stt.varint();
              else stt.skip(wt5);
            }
            if (!stt.ok) slow = true;
          } else {
            sp.skip(wt4);
          }
        }
        if (!sp.ok || !SigCache::cacheable(kind, code)) slow = true;
        p.name = reinterpret_cast<const uint8_t *>(name.data());
        p.nlen = (uint32_t)name.size();
        if (nd && !slow) {  // the signature name as the full path builds it
          p.noff = (uint32_t)arena.size();
          arena.append(name);
          for (size_t d = 0; d < nd && !slow; ++d) {
            char tag = '\x02';
            std::string_view val = dv[d];
            if (dt[d] == 2) {
              slow = true;
              break;
            }
            if (!dt[d]) {
              const Any *v = find_attr(b.rattrs, b.dims[d].name);
              if (!v) {
                arena += '\x03';
                continue;
              }
              if (v->type != kStr) {
                slow = true;
                break;
              }
              tag = '\x04', val = v->s;
            }
            const uint32_t n = (uint32_t)val.size();
            arena += tag;
            arena.append(reinterpret_cast<const char *>(&n), 4);
            arena.append(val);
          }
          p.nlen = (uint32_t)(arena.size() - p.noff);
        }
        p.slow = slow;
        if (!slow) {
          p.kind = kind, p.code = code, p.st = st, p.en = en;
          const bool has_tid = tid && tid_len == 16;
          p.w0 = has_tid ? rd64(tid) : 0, p.w1 = has_tid ? rd64(tid + 8) : 0;
          const std::string_view sn = nd ? std::string_view(arena.data() + p.noff, p.nlen) : name;
          p.sig = SigCache::hash(b.rhash, b.svc_id, sn, kind, code);
          if (b.own) b.cache.prefetch(p.sig);
          if (b.l2) b.l2->prefetch(p.sig);
        }
      }
      if (pend.empty()) return false;
    }
    for (const FastSpan &p : pend) {
      const SigCache::Rec *hit = nullptr;
      if (!p.slow) {
        const std::string_view sn = nd ? std::string_view(arena.data() + p.noff, p.nlen)
                                       : std::string_view(reinterpret_cast<const char *>(p.name), p.nlen);
        if (b.own) hit = b.cache.find(p.sig, b.rhash, b.svc_id, sn, p.kind, p.code);
        if (!hit) {
          b.own_misses += 1;
          if (b.l2) hit = b.l2->find(p.sig, b.rhash, b.svc_id, sn, p.kind, p.code);
        }
      }
      if (!hit) {
        ss.p = p.at;  // (a span's field was read whole: ss was fine there)
        return true;
      }
      if (p.en > b.out.max_end) b.out.max_end = p.en;
      const uint32_t kk = p.kind >= 0 && p.kind <= 7 ? (uint32_t)p.kind : 7u;
      const uint32_t cc = p.code >= 0 && p.code <= 3 ? (uint32_t)p.code : 3u;
      b.out.push(hit->sid, p.st, p.en, p.w0, p.w1, b.svc_id | (kk << 16) | (cc << 19));
      ++b.spans;
    }
  }
}
}  // namespace

struct Columnizer::Worker {
  Cols cols;
  SigCache cache;
  std::vector<FastSpan> pend;  // the batched path's spans and signature names
  std::string arena;
  std::vector<std::string_view> dim_val;
  std::vector<uint8_t> dim_type;
  bool own_cache_on = true;  // probe `cache` before the shared one (see columnize_batch)
  // spans decoded and own-cache misses (skipped probes included) since the
  // last decision; the hits are the difference (see columnize_batch)
  uint64_t own_spans = 0, own_misses = 0, batches = 0;
  std::vector<Attr> rattrs, sattrs, eattrs;
  std::vector<const Attr *> hv;
  std::string tmp, keystr, sname, service, evkey, sigbuf;
  std::vector<uint8_t> hbuf;
  std::vector<std::pair<const uint8_t *, const uint8_t *>> evs;  // the span's Event messages
  std::unordered_map<uint64_t, uint32_t> exl;                     // this request's exemplar candidates per series
};

struct Columnizer::Undo {
  std::vector<std::pair<uint64_t, std::string>> keys;
  std::vector<uint64_t> sids, resources;
  std::vector<std::string> services;
};

// threads 1..n-1 of a fork-join over one job; thread 0 is the caller.  A
// batch forks twice (decode, placement) and the host hands batches over
// back to back, so a worker first spins on the job epoch for a while
// (kSpinNs) before it blocks on the condition variable, and the caller spins
// the same way on the workers' completion: a blocked hand-over costs a futex
// wake per thread and per fork (~tens of microseconds for 15 threads).
struct Columnizer::Pool {
  static constexpr int64_t kSpinNs = 50000;
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable go, done;
  const std::function<void(unsigned)> *job = nullptr;
  std::atomic<uint64_t> epoch{0};
  std::atomic<unsigned> running{0};
  unsigned active = 0;
  std::atomic<bool> stop{false};

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  explicit Pool(unsigned n) {
    for (unsigned i = 1; i < n; ++i) th.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> l(m);
      stop.store(true);
    }
    go.notify_all();
    for (auto &t : th) t.join();
  }
  void loop(unsigned id) {
    uint64_t seen = 0;
    for (;;) {
      // spin, then block, until a new epoch (or stop)
      const int64_t t0 = now_ns();
      uint32_t k = 0;
      while (epoch.load(std::memory_order_acquire) == seen && !stop.load(std::memory_order_acquire)) {
        std::this_thread::yield();  // polite when the threads outnumber the cores
        if ((++k & 15u) == 0 && now_ns() - t0 > kSpinNs) {
          std::unique_lock<std::mutex> l(m);
          go.wait(l, [&] { return stop.load() || epoch.load() != seen; });
          break;
        }
      }
      if (stop.load(std::memory_order_acquire)) return;
      seen = epoch.load(std::memory_order_acquire);
      const auto *j = job;
      if (id < active) (*j)(id);
      if (running.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> l(m);  // the caller may be blocked on `done`
        done.notify_one();
      }
    }
  }
  void run(unsigned n, const std::function<void(unsigned)> &f) {
    job = &f;
    active = n;
    running.store((unsigned)th.size(), std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> l(m);
      epoch.fetch_add(1, std::memory_order_acq_rel);  // publishes job / active / running
    }
    go.notify_all();
    f(0);
    const int64_t t0 = now_ns();
    uint32_t k = 0;
    while (running.load(std::memory_order_acquire) != 0) {
      std::this_thread::yield();
      if ((++k & 15u) == 0 && now_ns() - t0 > kSpinNs) {
        std::unique_lock<std::mutex> l(m);
        done.wait(l, [&] { return running.load() == 0; });
        break;
      }
    }
  }
};

Columnizer::Columnizer(Options o) : opt_(std::move(o)), main_(new Worker) {}
Columnizer::~Columnizer() = default;

namespace {
// the connector's internal keys (connector.js OVERFLOW_KEY, EVENT_KEY_PREFIX)
const std::string kOverflowKey = std::string("\x01") + "otel.metric.overflow";
const std::string kEventKeyPrefix = std::string(1, '\x02') + "events" + std::string(1, '\0');
const std::string kNoKey;
bool span_key(const std::string &k) { return k.empty() || (k[0] != '\x01' && k[0] != '\x02'); }
}  // namespace

void Columnizer::learn(uint64_t rhash, const std::string &key, uint64_t sid) {
  auto &keys = res_keys_[rhash];
  if (keys.emplace(key, sid).second && span_key(key)) ++nspan_[rhash];
  keys[key] = sid;
  owner_[sid] = std::make_pair(rhash, key);
  ++gen_;
}

void Columnizer::accept_exemplars(Result &r) {
  if (r.exemplars.empty()) return;
  size_t k = 0;
  for (const SpanRef &x : r.exemplars) {
    uint32_t &c = ex_count_[x.sid];
    if (c < opt_.exemplars_max) {
      ++c;
      r.exemplars[k++] = x;
    }
  }
  r.exemplars.resize(k);
}

void Columnizer::remap(uint64_t from, uint64_t to) {
  for (size_t i = 0; i < buf_.n; ++i)
    if (buf_.key[i] == from) buf_.key[i] = to;
  ++gen_;
  auto o = owner_.find(from);
  if (o == owner_.end()) return;
  const auto who = o->second;
  owner_.erase(o);
  owner_[to] = who;
  res_keys_[who.first][who.second] = to;
}

// One request into `out`.  kShared (worker threads): the dictionaries are
// read-only, and anything not already in them -- a new resource, service or
// series -- or any failure returns false with nothing reported (the request is
// redone exclusively).  Exclusive: new entries go into the dictionaries and
// `undo`; false = res.status / res.error say why (the caller rolls back).
template <bool kShared>
bool Columnizer::run(const uint8_t *buf, size_t len, Worker &w, Cols &out, SigCache &cache, const SigCache *l2,
                     Result &res,
                     Undo *undo) {
  auto fail = [&](Result::Status st, const char *why) {
    if constexpr (!kShared) res.status = st, res.error = why;
    return false;
  };
  auto &rattrs = w.rattrs, &sattrs = w.sattrs;
  std::string &tmp = w.tmp, &keystr = w.keystr, &sname = w.sname, &service = w.service;
  auto &hbuf = w.hbuf;
  // the signature cache skips building the key string (a span with events
  // builds it anyway, for the event keys).  With dimensions the signature's
  // name is the span name followed by each dimension's string value (span
  // attribute, else resource attribute) or a marker for "absent": the key is
  // a function of exactly these, the service and the resource identity (a
  // non-string value takes the full path)
  const bool dims = !opt_.dims.empty();
  const bool own_on = w.own_cache_on;  // (fixed for the call: a local, not a load per span)
  w.exl.clear();
  PB req(buf, buf + len);
  uint32_t f;
  int wt;
  while (req.next(f, wt)) {
    if (f != 1 || wt != 2) {
      req.skip(wt);
      continue;
    }
    PB rs = req.sub();
    // pass 1: the Resource message (it may follow scope_spans on the wire)
    PB resource(nullptr, nullptr);
    bool has_resource = false;
    {
      PB scan = rs;
      uint32_t g;
      int wt2;
      while (scan.next(g, wt2)) {
        if (g == 1 && wt2 == 2) resource = scan.sub(), has_resource = true;
        else scan.skip(wt2);
      }
      if (!scan.ok) return fail(Result::kError, "malformed ResourceSpans");
    }
    rattrs.clear();
    if (has_resource) {
      PB r = resource;
      uint32_t g;
      int wt2;
      while (r.next(g, wt2)) {
        if (g == 1 && wt2 == 2) {
          Attr a;
          if (!parse_kv(r.sub(), a.key, a.val)) return fail(Result::kError, "malformed KeyValue");
          if (!valid_utf8(a.key)) return fail(Result::kFallback, "non-UTF-8 attribute key");
          rattrs.push_back(a);
        } else {
          r.skip(wt2);
        }
      }
      if (!r.ok) return fail(Result::kError, "malformed Resource");
    }
    dedupe_last(rattrs);
    const Any *svc = find_attr(rattrs, "service.name");
    if (!svc) continue;  // A1: a resource without service.name contributes nothing
    service.clear();
    if (svc->type == kStr) {
      if (!valid_utf8(svc->s)) return fail(Result::kFallback, "non-UTF-8 service.name");
      service.assign(svc->s);
    }
    // resource identity (keys.js resourceHash over the key attributes)
    auto &hv = w.hv;
    hv.clear();
    for (const Attr &a : rattrs) {
      if (opt_.key_attributes.empty() ||
          std::find(opt_.key_attributes.begin(), opt_.key_attributes.end(), a.key) != opt_.key_attributes.end())
        hv.push_back(&a);
    }
    std::sort(hv.begin(), hv.end(), [](const Attr *x, const Attr *y) { return x->key < y->key; });
    hbuf.clear();
    for (const Attr *a : hv) {
      if (const Keyable k = as_string(a->val, tmp); k != Keyable::kYes)
        return k == Keyable::kTooDeep ? fail(Result::kError, "attribute value nested too deeply")
                                      : fail(Result::kFallback, "resource attribute not keyable natively");
      hbuf.insert(hbuf.end(), a->key.begin(), a->key.end());
      hbuf.push_back(0);
      hbuf.insert(hbuf.end(), tmp.begin(), tmp.end());
      hbuf.push_back(0);
      const char *tag = kTypeTag[a->val.type];
      hbuf.insert(hbuf.end(), tag, tag + std::strlen(tag));
      hbuf.push_back(1);
    }
    const uint64_t rhash = xxh64(hbuf.data(), hbuf.size(), 0);
    auto rit = res_keys_.find(rhash);
    if (rit == res_keys_.end()) {
      if constexpr (kShared) return false;
      rit = res_keys_.emplace(rhash, std::unordered_map<std::string, uint64_t>{}).first;
      undo->resources.push_back(rhash);
      res.new_resources.push_back({rhash, has_resource ? (int64_t)(resource.p - buf) : -1,
                                   has_resource ? (uint32_t)(resource.end - resource.p) : 0u});
    }
    auto &keys = rit->second;
    res.resources.push_back(rhash);
    const int64_t res_off = has_resource ? (int64_t)(resource.p - buf) : -1;
    const uint32_t res_len = has_resource ? (uint32_t)(resource.end - resource.p) : 0u;
    // a new series id for `key` of this resource (exclusive calls only): seed
    // 0, 1, ... until the id is neither 0 (reserved) nor another series'
    auto intern = [&](const std::string &key) -> uint64_t {
      hbuf.resize(8 + key.size());
      std::memcpy(hbuf.data(), &rhash, 8);
      std::memcpy(hbuf.data() + 8, key.data(), key.size());
      uint64_t id = 0;
      for (uint64_t seed = 0;; ++seed) {
        id = (opt_.test_collide_seed0 && seed == 0) ? 42 : xxh64(hbuf.data(), hbuf.size(), seed);
        if (id == 0) continue;
        auto o = owner_.find(id);
        if (o == owner_.end()) {
          owner_.emplace(id, std::make_pair(rhash, key));
          undo->sids.push_back(id);
          break;
        }
        if (o->second.first == rhash && o->second.second == key) break;
      }
      keys.emplace(key, id);
      undo->keys.emplace_back(rhash, key);
      if (span_key(key)) ++nspan_[rhash];
      return id;
    };
    uint32_t svc_id;
    if constexpr (kShared) {
      auto it = services_.find(service);
      if (it == services_.end()) return false;
      svc_id = it->second;
    } else {
      bool svc_new = false;
      svc_id = service_id(service, &svc_new);
      if (svc_new) {
        undo->services.push_back(service);
        res.new_services.emplace_back(service, svc_id);
      }
    }

    // pass 2: scope_spans -> spans.  Batched (see the span loop) when the
    // lookups will miss the CPU caches: this thread's own cache is not probed
    // (a high-cardinality stream, see columnize_batch) or holds more
    // signatures than a core's caches do
    const bool batched = !opt_.events && !opt_.exemplars && (!own_on || cache.size() > kBatchAbove || opt_.test_batched);
    PB scan = rs;
    uint32_t g;
    int wt2;
    while (scan.next(g, wt2)) {
      if (g != 2 || wt2 != 2) {
        scan.skip(wt2);
        continue;
      }
      PB ss = scan.sub();
      uint32_t h;
      int wt3;
      // One loop: in batched mode batch_hits emits the spans whose signature
      // the caches hold and stops at the first it cannot resolve, with the
      // scope's parser back at that span; the full path below takes that one
      // span, then the batched mode resumes.  (Only copies of the parser go
      // to batch_hits, so the plain loop's state stays in registers.)
      BatchScope bs{w.pend, w.arena, w.dim_val, w.dim_type, own_on, opt_.dims, rattrs, rhash, svc_id,
                    cache, l2, out, res.spans, w.own_misses};
      for (;;) {
        if (batched) {
          PB bss = ss;
          const bool more = batch_hits(bs, bss);
          ss = bss;
          if (!more) break;
        }
        if (!ss.next(h, wt3)) break;
        if (h != 2 || wt3 != 2) {
          ss.skip(wt3);
          continue;
        }
        PB sp = ss.sub();
        // the full path: one span, any configuration
        const uint8_t *span_begin = sp.p, *span_end = sp.end;
        const uint8_t *tid = nullptr, *spid = nullptr;
        size_t tid_len = 0, spid_len = 0;
        std::string_view name;
        int32_t kind = 0, code = 0;
        uint64_t st = 0, en = 0;
        sattrs.clear();
        if (opt_.events) w.evs.clear();
        uint32_t k;
        int wt4;
        while (sp.next(k, wt4)) {
          if (k == 1 && wt4 == 2) {
            const std::string_view t = sp.str();
            tid = reinterpret_cast<const uint8_t *>(t.data());
            tid_len = t.size();
          } else if (k == 2 && wt4 == 2 && opt_.exemplars) {
            const std::string_view t = sp.str();
            spid = reinterpret_cast<const uint8_t *>(t.data());
            spid_len = t.size();
          } else if (k == 5 && wt4 == 2) {
            name = sp.str();
          } else if (k == 6 && wt4 == 0) {
            kind = (int32_t)(uint32_t)sp.varint();
          } else if (k == 7 && wt4 == 1) {
            st = sp.fixed64();
          } else if (k == 8 && wt4 == 1) {
            en = sp.fixed64();
          } else if (k == 9 && wt4 == 2 && !opt_.dims.empty()) {
            Attr a;
            if (!parse_kv(sp.sub(), a.key, a.val)) return fail(Result::kError, "malformed KeyValue");
            sattrs.push_back(a);
          } else if (k == 11 && wt4 == 2 && opt_.events) {
            const PB ev = sp.sub();
            w.evs.emplace_back(ev.p, ev.end);
          } else if (k == 15 && wt4 == 2) {
            PB stt = sp.sub();
            uint32_t m;
            int wt5;
            code = 0;  // a later Status message replaces an earlier one
            while (stt.next(m, wt5)) {
              if (m == 3 && wt5 == 0) code = (int32_t)(uint32_t)stt.varint();
              else stt.skip(wt5);
            }
            if (!stt.ok) return fail(Result::kError, "malformed Status");
          } else {
            sp.skip(wt4);
          }
        }
        if (!sp.ok) return fail(Result::kError, "malformed Span");
        uint64_t sid;
        uint64_t sig = 0;
        const SigCache::Rec *hit = nullptr;
        std::string_view signame = name;
        bool use_cache = true;
        if (dims) {
          std::string &sb = w.sigbuf;
          sb.assign(name);
          for (const Dim &d : opt_.dims) {
            const Any *v = find_attr(sattrs, d.name);
            char tag = '\x02';
            if (!v) v = find_attr(rattrs, d.name), tag = '\x04';
            if (!v) {
              sb += '\x03';
              continue;
            }
            if (v->type != kStr) {
              use_cache = false;
              break;
            }
            const uint32_t n = (uint32_t)v->s.size();
            sb += tag;
            sb.append(reinterpret_cast<const char *>(&n), 4);
            sb.append(v->s);
          }
          signame = sb;
        }
        bool l2_hit = false;  // (an entry of the shared cache is read only here)
        if (use_cache && SigCache::cacheable(kind, code)) {
          sig = SigCache::hash(rhash, svc_id, signame, kind, code);
          if (own_on) hit = cache.find(sig, rhash, svc_id, signame, kind, code);
          if (!hit) {
            w.own_misses += 1;  // (rare where the own cache pays: one store per miss)
            if (l2 && (hit = l2->find(sig, rhash, svc_id, signame, kind, code))) l2_hit = true;
          }
        }
        // key = buildKey, into keystr (0 = built; else the failure to return)
        auto build_key = [&]() -> int {
          if (!valid_utf8(name)) return 1;
          sname = apply_rules(opt_.rules, std::string(name));
          keystr.clear();
          bool first = true;
          auto part = [&](std::string_view s) {
            if (!first) keystr += '\0';
            first = false;
            keystr += s;
          };
          if (!opt_.ex_service) part(service);
          if (!opt_.ex_name) part(sname);
          if (!opt_.ex_kind) part(kind >= 0 && kind < 6 ? kKindStr[kind] : "");
          if (!opt_.ex_status) part(code >= 0 && code < 3 ? kStatusStr[code] : "");
          for (const Dim &d : opt_.dims) {
            const Any *v = find_attr(sattrs, d.name);
            if (!v) v = find_attr(rattrs, d.name);
            if (v) {
              if (const Keyable kb = as_string(*v, tmp); kb != Keyable::kYes) return kb == Keyable::kTooDeep ? 2 : 3;
            } else if (d.has_default) {
              tmp = d.def;
            } else {
              continue;  // A5: missing optional dimension, no separator
            }
            keystr += '\0';
            keystr += tmp;
          }
          return 0;
        };
        auto key_fail = [&](int why) {
          return why == 1   ? fail(Result::kFallback, "non-UTF-8 span name")
                 : why == 2 ? fail(Result::kError, "attribute value nested too deeply")
                            : fail(Result::kFallback, "dimension value not keyable natively");
        };
        if (hit) {
          sid = hit->sid;
          if (opt_.events && !w.evs.empty()) {  // the event keys extend the span key: kept in the entry
            const std::string &hk = (l2_hit ? l2 : &cache)->rec_entry(hit).key;
            if (!hk.empty()) keystr = hk;
            else if (const int why = build_key()) return key_fail(why);
          }
        } else {
          if (const int why = build_key()) return key_fail(why);
          auto kit = keys.find(keystr);
          bool overflow = false;
          if (kit != keys.end()) {
            sid = kit->second;
          } else {
            if constexpr (kShared) return false;
            auto ns = nspan_.find(rhash);
            if (opt_.card_limit && ns != nspan_.end() && ns->second >= opt_.card_limit) {
              // aggregation_cardinality_limit: the resource's overflow series
              overflow = true;
              auto ov = keys.find(kOverflowKey);
              if (ov != keys.end()) {
                sid = ov->second;
              } else {
                sid = intern(kOverflowKey);
                res.new_series.push_back(
                    {sid, rhash, (uint32_t)(span_begin - buf), (uint32_t)(span_end - span_begin), res_off, res_len});
              }
            } else {
              sid = intern(keystr);
              res.new_series.push_back(
                  {sid, rhash, (uint32_t)(span_begin - buf), (uint32_t)(span_end - span_begin), res_off, res_len});
            }
          }
          // (an overflowed key is decided again each time: the count it met may change)
          if (use_cache && !overflow)
            cache.insert(sig, rhash, svc_id, signame, kind, code, sid, opt_.events ? keystr : kNoKey);
        }
        // candidates; accept_exemplars keeps the interval's first ones.  A
        // series seen full this interval is marked in its signature-cache
        // entry, so its later spans cost no lookup.
        if (opt_.exemplars && !(hit && (l2_hit ? l2 : &cache)->rec_entry(hit).ex_full == ex_gen_)) {
          auto ex = ex_count_.find(sid);
          const uint32_t taken = ex == ex_count_.end() ? 0u : ex->second;
          if (taken < opt_.exemplars_max) {
            uint32_t &mine = w.exl[sid];
            if (taken + mine < opt_.exemplars_max) {
              ++mine;
              SpanRef x{sid, (uint32_t)(span_begin - buf), (uint32_t)(span_end - span_begin)};
              if (tid && tid_len == 16 && spid && spid_len == 8) {
                x.ids_ok = true;
                std::memcpy(x.ids, tid, 16);
                std::memcpy(x.ids + 16, spid, 8);
                x.start = st, x.end = en;
              }
              res.exemplars.push_back(x);
            }
          } else if (hit) {
            if (!l2_hit) cache.rec_entry(hit).ex_full = ex_gen_;
          }
        }
        if (en > out.max_end) out.max_end = en;
        const bool has_tid = tid && tid_len == 16;
        const uint32_t kk = kind >= 0 && kind <= 7 ? (uint32_t)kind : 7u;
        const uint32_t cc = code >= 0 && code <= 3 ? (uint32_t)code : 3u;
        out.push(sid, st, en, has_tid ? rd64(tid) : 0, has_tid ? rd64(tid + 8) : 0, svc_id | (kk << 16) | (cc << 19));
        ++res.spans;
        // events.enabled: one record per event, keyed by the span key and the
        // event dimensions (connector.js _eventId), counted as a span of
        // duration 0 with an out-of-range service id (no sketch)
        for (uint32_t ei = 0; opt_.events && ei < (uint32_t)w.evs.size(); ++ei) {
          auto &eattrs = w.eattrs;
          eattrs.clear();
          PB ev(w.evs[ei].first, w.evs[ei].second);
          uint32_t m;
          int wt5;
          while (ev.next(m, wt5)) {
            if (m == 3 && wt5 == 2) {
              Attr a;
              if (!parse_kv(ev.sub(), a.key, a.val)) return fail(Result::kError, "malformed KeyValue");
              eattrs.push_back(a);
            } else {
              ev.skip(wt5);
            }
          }
          if (!ev.ok) return fail(Result::kError, "malformed Span.Event");
          dedupe_last(eattrs);
          std::string &ek = w.evkey;
          ek.assign(kEventKeyPrefix);
          ek += keystr;
          for (const Dim &d : opt_.event_dims) {
            const Any *v = find_attr(eattrs, d.name);
            if (v) {
              if (const Keyable kb = as_string(*v, tmp); kb != Keyable::kYes)
                return kb == Keyable::kTooDeep ? fail(Result::kError, "attribute value nested too deeply")
                                               : fail(Result::kFallback, "event dimension not keyable natively");
            } else if (d.has_default) {
              tmp = d.def;
            } else {
              continue;
            }
            ek += '\0';
            ek += tmp;
          }
          uint64_t esid;
          auto eit = keys.find(ek);
          if (eit != keys.end()) {
            esid = eit->second;
          } else {
            if constexpr (kShared) return false;
            esid = intern(ek);
            res.new_event_series.push_back(
                {esid, rhash, (uint32_t)(span_begin - buf), (uint32_t)(span_end - span_begin), ei, res_off, res_len});
          }
          out.push(esid, 0, 0, 0, 0, 0xFFFFu);
          ++res.event_records;
        }
            }
      if (!ss.ok) return fail(Result::kError, "malformed ScopeSpans");
    }
    if (!scan.ok) return fail(Result::kError, "malformed ResourceSpans");
  }
  if (!req.ok) return fail(Result::kError, "malformed ExportTraceServiceRequest");
  return true;
}

Result Columnizer::columnize(const uint8_t *buf, size_t len) {
  Result r = columnize_into(buf, len, buf_);
  cache_.drop_fresh();  // (one thread: no shared cache to fill)
  accept_exemplars(r);
  return r;
}

Result Columnizer::columnize_into(const uint8_t *buf, size_t len, Cols &out) {
  if (cache_.gen != gen_) cache_.clear(), cache_.gen = gen_;
  // the second level too: a remap or forget since the last batch filled it
  // (both bump gen_) may have changed the series an entry names
  if (shared_.gen != gen_) shared_.clear(), shared_.gen = gen_;
  Result res;
  Undo undo;
  const size_t n0 = out.size();
  const uint64_t max0 = out.max_end;
  if (run<false>(buf, len, *main_, out, cache_, &shared_, res, &undo)) return res;
  // all or nothing: drop this call's columns and dictionary entries
  out.truncate(n0);
  out.max_end = max0;
  for (auto &k : undo.keys) {
    auto it = res_keys_.find(k.first);
    if (it != res_keys_.end()) it->second.erase(k.second);
    if (span_key(k.second)) {
      auto ns = nspan_.find(k.first);
      if (ns != nspan_.end() && ns->second) --ns->second;
    }
  }
  for (uint64_t h : undo.resources) res_keys_.erase(h);
  for (uint64_t sid : undo.sids) owner_.erase(sid);
  for (auto &s : undo.services) services_.erase(s);
  cache_.clear();  // it may name series this call made
  Result r;
  r.status = res.status;
  r.error = res.error;
  return r;
}

BatchResult Columnizer::columnize_batch(const uint8_t *const *bufs, const size_t *lens, size_t n) {
  BatchResult br;
  const unsigned T = (unsigned)std::min<size_t>(std::max(1u, opt_.threads), n);
  if (T <= 1) {
    for (size_t i = 0; i < n; ++i) {
      br.results.push_back(columnize(bufs[i], lens[i]));
      if (br.results.back().status == Result::kFallback) {
        br.done = i + 1;
        return br;
      }
    }
    br.done = n;
    return br;
  }
  struct Slot {
    const Cols *src = nullptr;
    bool ok = false;
    size_t off = 0, cnt = 0, dst = 0;
    uint64_t max_end = 0;
    Result r;
  };
  std::vector<Slot> slots(n);
  while (workers_.size() < opt_.threads) workers_.emplace_back(new Worker);
  if (!pool_) pool_.reset(new Pool(opt_.threads));
  // the threads' own caches stay small (a high-cardinality stream would give
  // every thread a copy of every series); the shared one holds them all
  constexpr size_t kOwnCacheMax = 1u << 15;
  if (shared_.gen != gen_) shared_.clear(), shared_.gen = gen_;
  for (auto &w : workers_) {
    // a thread's own cache pays only when its hot set fits it: past ~4 k
    // spans with fewer than 1 in 8 answered there (a high-cardinality
    // stream), it is not probed (its inserts still feed the shared cache);
    // every 32nd batch probes it again to re-sample.  (The spans are counted
    // from the thread's columns of the last batch, the misses in run.)
    w->own_spans += w->cols.size();
    w->cols.clear();
    if (w->cache.gen != gen_ || w->cache.size() > kOwnCacheMax) w->cache.clear(), w->cache.gen = gen_;
    w->batches += 1;
    if (w->own_spans >= 4096) {
      w->own_cache_on = 8 * (w->own_spans - std::min(w->own_misses, w->own_spans)) >= w->own_spans;
      w->own_spans = w->own_misses = 0;
    }
    if (!w->own_cache_on && (w->batches & 31u) == 0) w->own_cache_on = true, w->own_spans = w->own_misses = 0;
  }
  using clk = std::chrono::steady_clock;
  const auto ns_since = [](clk::time_point t) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t).count();
  };
  auto t_ph = clk::now();
  // phase 1: decode in parallel against the dictionaries as they stand
  std::atomic<size_t> next{0};
  const std::function<void(unsigned)> decode = [&](unsigned wid) {
    Worker &w = *workers_[wid];
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) {
      Slot &s = slots[i];
      s.src = &w.cols;
      s.off = w.cols.size();
      w.cols.max_end = 0;
      try {
        s.ok = run<true>(bufs[i], lens[i], w, w.cols, w.cache, &shared_, s.r, nullptr);
      } catch (...) {  // e.g. bad_alloc: redone (and reported) on the caller's thread
        s.ok = false;
      }
      if (!s.ok) {
        w.cols.truncate(s.off);
        s.r = Result();
        continue;
      }
      s.cnt = w.cols.size() - s.off;
      s.max_end = w.cols.max_end;
    }
  };
  pool_->run(T, decode);
  br.ns_decode = ns_since(t_ph);
  t_ph = clk::now();
  // phase 2, in request order: what phase 1 could not take is redone exclusively
  excl_.clear();
  size_t taken = n, total = 0;
  for (size_t i = 0; i < n; ++i) {
    Slot &s = slots[i];
    if (!s.ok) {
      s.src = &excl_;
      s.off = excl_.size();
      excl_.max_end = 0;
      s.r = columnize_into(bufs[i], lens[i], excl_);
      s.cnt = excl_.size() - s.off;
      s.max_end = excl_.max_end;
    }
    accept_exemplars(s.r);
    s.dst = buf_.size() + total;
    total += s.cnt;
    if (s.max_end > buf_.max_end) buf_.max_end = s.max_end;
    if (s.r.status == Result::kFallback) {
      taken = i + 1;
      break;
    }
  }
  br.ns_commit = ns_since(t_ph);
  t_ph = clk::now();
  // phase 3: every request's columns to its place in the buffer, in parallel
  const size_t base = buf_.size();
  buf_.reserve(base + total);
  buf_.n = base + total;
  next = 0;
  const std::function<void(unsigned)> place = [&](unsigned) {
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < taken;) {
      const Slot &s = slots[i];
      if (!s.cnt) continue;
      const Cols &c = *s.src;
      std::memcpy(&buf_.key[s.dst], &c.key[s.off], s.cnt * 8);
      std::memcpy(&buf_.start[s.dst], &c.start[s.off], s.cnt * 8);
      std::memcpy(&buf_.end[s.dst], &c.end[s.off], s.cnt * 8);
      std::memcpy(&buf_.w0[s.dst], &c.w0[s.off], s.cnt * 8);
      std::memcpy(&buf_.w1[s.dst], &c.w1[s.off], s.cnt * 8);
      std::memcpy(&buf_.meta[s.dst], &c.meta[s.off], s.cnt * 4);
    }
  };
  pool_->run(T, place);
  br.ns_place = ns_since(t_ph);
  // the signatures the threads resolved this batch -> the shared cache
  const auto merge = [&](const SigCache::Entry &e, std::string_view name) {
    if (!shared_.find(e.h, e.rhash, e.svc, name, e.kind, e.code))
      shared_.insert(e.h, e.rhash, e.svc, name, e.kind, e.code, e.sid, e.key);
  };
  for (auto &w : workers_) w->cache.take_fresh(merge);
  if (cache_.gen == gen_) cache_.take_fresh(merge);  // (the requests redone on this thread)
  shared_.drop_fresh();
  br.results.reserve(taken);
  for (size_t i = 0; i < taken; ++i) br.results.push_back(std::move(slots[i].r));
  br.done = taken;
  return br;
}

}  // namespace otlpcol
