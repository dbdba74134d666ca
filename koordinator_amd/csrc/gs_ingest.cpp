// gs_ingest.cpp — ingest decoders: the annotation and label text the hot-path plugins read,
// decoded into the ABI structs on the host before it crosses PCIe as SoA delta rows. Each decoder restates the
// reference function it replaces (file:line in include/gpuscore.h): Go encoding/json into the same Go types,
// k8s resource.Quantity, time.ParseDuration, cpuset.Parse. Errors follow the reference's: where a plugin
// ignores a malformed annotation the decoder records "absent", where it fails the decoder does too.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/gpuscore.h"

namespace {

// ---- a small JSON DOM (RFC 8259), enough for encoding/json.Unmarshal into the reference's types ----
struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  std::string text;                                      // NUM: the literal; STR: the decoded string
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;         // insertion order; Go keeps the last duplicate
  const JVal* get(const char* k) const {
    const JVal* r = nullptr;
    for (const auto& kv : obj)
      if (kv.first == k) r = &kv.second;
    return r;
  }
};

struct JParser {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) < n || memcmp(p, s, n) != 0) return false;
    p += n;
    return true;
  }
  static void utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 63)); }
    else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63)); }
    else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 63)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63)); }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    *v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      *v <<= 4;
      if (c >= '0' && c <= '9') *v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') *v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') *v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    return true;
  }
  bool str(std::string& o) {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      unsigned char c = (unsigned char)*p;
      if (c < 0x20) return false;
      if (c != '\\') { o += (char)c; ++p; continue; }
      if (++p >= e) return false;
      char x = *p++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t u;
          if (!hex4(&u)) return false;
          if (u >= 0xD800 && u < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
            else { p = save; u = 0xFFFD; }
          } else if (u >= 0xD800 && u < 0xE000) {
            u = 0xFFFD;
          }
          utf8(o, u);
          break;
        }
        default: return false;
      }
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  bool num(std::string& o) {
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p >= e) return false;
    if (*p == '0') ++p;
    else if (*p >= '1' && *p <= '9') while (p < e && *p >= '0' && *p <= '9') ++p;
    else return false;
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    o.assign(s, p);
    return true;
  }
  bool value(JVal& v, int depth) {
    if (depth > 64) return false;
    ws();
    if (p >= e) return false;
    char c = *p;
    if (c == '{') {
      ++p;
      v.kind = JVal::OBJ;
      ws();
      if (p < e && *p == '}') { ++p; return true; }
      for (;;) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (p >= e || *p != ':') return false;
        ++p;
        JVal x;
        if (!value(x, depth + 1)) return false;
        v.obj.emplace_back(std::move(k), std::move(x));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; return true; }
        return false;
      }
    }
    if (c == '[') {
      ++p;
      v.kind = JVal::ARR;
      ws();
      if (p < e && *p == ']') { ++p; return true; }
      for (;;) {
        JVal x;
        if (!value(x, depth + 1)) return false;
        v.arr.push_back(std::move(x));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; return true; }
        return false;
      }
    }
    if (c == '"') { v.kind = JVal::STR; return str(v.text); }
    if (lit("true")) { v.kind = JVal::BOOL; v.b = true; return true; }
    if (lit("false")) { v.kind = JVal::BOOL; v.b = false; return true; }
    if (lit("null")) { v.kind = JVal::NUL; return true; }
    v.kind = JVal::NUM;
    return num(v.text);
  }
};

bool parse_json(const char* s, JVal* out) {
  if (!s) return false;
  JParser jp{s, s + strlen(s)};
  if (!jp.value(*out, 0)) return false;
  jp.ws();
  return jp.p == jp.e;
}

// encoding/json into int64: an integer literal in range (no fraction or exponent)
bool json_int64(const JVal& v, int64_t* out) {
  if (v.kind != JVal::NUM) return false;
  for (char c : v.text)
    if (c == '.' || c == 'e' || c == 'E') return false;
  errno = 0;
  char* end = nullptr;
  long long x = strtoll(v.text.c_str(), &end, 10);
  if (errno || *end) return false;
  *out = x;
  return true;
}
// encoding/json into int32
bool json_int32(const JVal& v, int32_t* out) {
  int64_t x;
  if (!json_int64(v, &x) || x < INT32_MIN || x > INT32_MAX) return false;
  *out = (int32_t)x;
  return true;
}
// encoding/json into float64 (strtod is correctly rounded, as strconv.ParseFloat)
bool json_float64(const JVal& v, double* out) {
  if (v.kind != JVal::NUM) return false;
  errno = 0;
  char* end = nullptr;
  double x = strtod(v.text.c_str(), &end);
  if (*end || (errno == ERANGE && std::isinf(x))) return false;
  *out = x;
  return true;
}

const char* find_kv(const gs_kv* kv, uint32_t n, const char* key) {
  const char* r = nullptr;
  for (uint32_t i = 0; i < n; ++i)
    if (kv[i].key && strcmp(kv[i].key, key) == 0) r = kv[i].value ? kv[i].value : "";
  return r;
}

// ---- [upstream] k8s.io/apimachinery@v0.24.15 resource.ParseQuantity, Value() / MilliValue() (round up) ----
// value = mantissa x 10^e10 x 2^e2, exact over __int128; ceil(value x 10^scale10).
int quantity_scaled(const char* s, int scale10, int64_t* out) {
  if (!s) return GS_EINVAL;
  const char* p = s;
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
  __int128 m = 0;
  int digits = 0, frac = 0;
  bool any = false;
  while (*p >= '0' && *p <= '9') {
    if (m != 0 || *p != '0') ++digits;
    if (digits > 36) return GS_EUNSUPPORTED;
    m = m * 10 + (*p - '0');
    ++p;
    any = true;
  }
  if (*p == '.') {
    ++p;
    while (*p >= '0' && *p <= '9') {
      if (m != 0 || *p != '0') ++digits;
      if (digits > 36) return GS_EUNSUPPORTED;
      m = m * 10 + (*p - '0');
      ++frac;
      ++p;
      any = true;
    }
  }
  if (!any) return GS_EINVAL;
  int e10 = -frac, e2 = 0;
  // suffix: binarySI Ki..Ei, decimalSI n u m "" k M G T P E, or a decimal exponent e<int> / E<int>
  const std::string suf(p);
  static const std::map<std::string, int> bin = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  static const std::map<std::string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                 {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  auto bi = bin.find(suf);
  auto di = dec.find(suf);
  if (bi != bin.end()) e2 = bi->second;
  else if (di != dec.end()) e10 += di->second;
  else if ((suf[0] == 'e' || suf[0] == 'E') && suf.size() > 1) {
    const char* q = suf.c_str() + 1;
    bool en = false;
    if (*q == '+' || *q == '-') { en = *q == '-'; ++q; }
    if (!*q) return GS_EINVAL;
    int x = 0;
    for (; *q; ++q) {
      if (*q < '0' || *q > '9') return GS_EINVAL;
      x = x * 10 + (*q - '0');
      if (x > 1000) return GS_EUNSUPPORTED;
    }
    e10 += en ? -x : x;
  } else {
    return GS_EINVAL;
  }
  e10 += scale10;
  if (m == 0) { *out = 0; return GS_OK; }
  // A negative quantity takes apimachinery's int64Amount or inf.Dec path by its digits and suffix, and the two
  // round an inexact Value() differently (away from zero vs truncate-then-add-one); resource requests, allocatable
  // and the annotations decoded here are non-negative in every valid object, so a negative one is refused
  // instead of being rounded by one rule for both paths.
  if (neg) return GS_EUNSUPPORTED;
  const __int128 lim = (__int128)INT64_MAX;
  for (int i = 0; i < e2; ++i) { m *= 2; if (m > lim * 1000) return GS_EUNSUPPORTED; }
  __int128 q;
  if (e10 >= 0) {
    q = m;
    for (int i = 0; i < e10; ++i) { q *= 10; if (q > lim) return GS_EUNSUPPORTED; }
  } else if (-e10 > 36) {
    *out = 1;   // 0 < value < 1 after scaling: ceil is 1
    return GS_OK;
  } else {
    __int128 d = 1;
    for (int i = 0; i < -e10; ++i) d *= 10;
    q = m / d;
    if (m % d != 0) q += 1;   // ceil
  }
  if (q > lim) return GS_EUNSUPPORTED;
  *out = (int64_t)q;
  return GS_OK;
}

// Quantity.UnmarshalJSON: a JSON string or a bare number literal (null = zero)
int quantity_json(const JVal& v, int scale10, int64_t* out) {
  if (v.kind == JVal::STR || v.kind == JVal::NUM) {
    std::string t = v.text;
    size_t a = t.find_first_not_of(" \t\n\r"), b = t.find_last_not_of(" \t\n\r");
    t = a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
    return quantity_scaled(t.c_str(), scale10, out);
  }
  if (v.kind == JVal::NUL) { *out = 0; return GS_OK; }
  return GS_EINVAL;
}

// [upstream] Go time.ParseDuration (int64 ns; fractions through float64 as Go does)
bool parse_duration(const std::string& s0, int64_t* out) {
  const char* p = s0.c_str();
  bool neg = false;
  if (*p == '-' || *p == '+') { neg = *p == '-'; ++p; }
  if (strcmp(p, "0") == 0) { *out = 0; return true; }
  if (!*p) return false;
  uint64_t d = 0;
  while (*p) {
    if (!(*p == '.' || (*p >= '0' && *p <= '9'))) return false;
    uint64_t v = 0, f = 0;
    double scale = 1;
    bool pre = false, post = false;
    while (*p >= '0' && *p <= '9') {
      if (v > (UINT64_MAX >> 1) / 10) return false;
      v = v * 10 + (uint64_t)(*p - '0');
      ++p;
      pre = true;
    }
    if (*p == '.') {
      ++p;
      bool overflow = false;
      while (*p >= '0' && *p <= '9') {
        if (!overflow) {
          if (f > (UINT64_MAX >> 1) / 10) overflow = true;
          else { f = f * 10 + (uint64_t)(*p - '0'); scale *= 10; }
        }
        ++p;
        post = true;
      }
    }
    if (!pre && !post) return false;
    const char* u0 = p;
    while (*p && *p != '.' && !(*p >= '0' && *p <= '9')) ++p;
    const std::string unit(u0, p);
    uint64_t mul;
    if (unit == "ns") mul = 1;
    else if (unit == "us" || unit == "\xC2\xB5s" || unit == "\xCE\xBCs") mul = 1000;
    else if (unit == "ms") mul = 1000000;
    else if (unit == "s") mul = 1000000000ull;
    else if (unit == "m") mul = 60ull * 1000000000ull;
    else if (unit == "h") mul = 3600ull * 1000000000ull;
    else return false;
    if (v > (uint64_t)INT64_MAX / mul) return false;
    v *= mul;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)mul / scale));
      if (v > (uint64_t)INT64_MAX) return false;
    }
    d += v;
    if (d > (uint64_t)INT64_MAX) return false;
  }
  *out = neg ? -(int64_t)d : (int64_t)d;
  return true;
}

// map[corev1.ResourceName]int64 -> cpu / memory values + GS_USAGE_* key mask
bool thresholds_map(const JVal* v, int64_t vals[2], uint32_t* mask) {
  vals[0] = vals[1] = 0;
  *mask = 0;
  if (!v || v->kind == JVal::NUL) return true;
  if (v->kind != JVal::OBJ) return false;
  for (const auto& kv : v->obj) {
    int64_t x;
    if (!json_int64(kv.second, &x)) return false;
    if (kv.first == "cpu") { vals[0] = x; *mask |= GS_USAGE_CPU; }
    else if (kv.first == "memory") { vals[1] = x; *mask |= GS_USAGE_MEMORY; }
    else *mask |= GS_USAGE_OTHER;
  }
  return true;
}

int agg_type(const std::string& s, int32_t* out) {
  if (s.empty()) *out = GS_AGG_NONE;
  else if (s == "avg") *out = GS_AGG_AVG;
  else if (s == "p50") *out = GS_AGG_P50;
  else if (s == "p90") *out = GS_AGG_P90;
  else if (s == "p95") *out = GS_AGG_P95;
  else if (s == "p99") *out = GS_AGG_P99;
  else return GS_EUNSUPPORTED;
  return GS_OK;
}


// NodeReservation (apis/extension/node_reservation.go:37-44) as encoding/json.Unmarshal fills it from the annotation
// node.koordinator.sh/reservation (GetNodeReservation, :59-68): present = the annotation is non-empty and decodes.
struct NodeRsv {
  bool present = false;
  std::vector<std::pair<std::string, const JVal*>> resources;   // ResourceList entries (Quantity JSON)
  std::string reserved_cpus, apply_policy;
  JVal doc;
};
bool node_reservation(const gs_kv* kv, uint32_t n, NodeRsv* r) {
  const char* s = find_kv(kv, n, "node.koordinator.sh/reservation");
  if (!s || !*s) return true;                       // absent / "": nil reservation
  if (!parse_json(s, &r->doc)) return false;
  if (r->doc.kind == JVal::NUL) { r->present = true; return true; }   // "null": an empty reservation
  if (r->doc.kind != JVal::OBJ) return false;
  if (const JVal* res = r->doc.get("resources")) {
    if (res->kind == JVal::OBJ) {
      for (const auto& e : res->obj) {
        int64_t x;
        const int rc = quantity_json(e.second, e.first == "cpu" ? 3 : 0, &x);
        if (rc == GS_EINVAL) return false;          // Quantity.UnmarshalJSON error
        r->resources.emplace_back(e.first, &e.second);
      }
    } else if (res->kind != JVal::NUL) {
      return false;
    }
  }
  for (const char* f : {"reservedCPUs", "applyPolicy"}) {
    const JVal* v = r->doc.get(f);
    if (!v || v->kind == JVal::NUL) continue;
    if (v->kind != JVal::STR) return false;
    (f[0] == 'r' ? r->reserved_cpus : r->apply_policy) = v->text;
  }
  r->present = true;
  return true;
}

int res_slot(const std::string& name) {   // gs_resource slot of a resource name, -1: none in gs_node
  static const char* names[7] = {"cpu", "memory", "ephemeral-storage", "kubernetes.io/batch-cpu",
                                          "kubernetes.io/batch-memory", "kubernetes.io/mid-cpu",
                                          "kubernetes.io/mid-memory"};
  for (int i = 0; i < 7; ++i)
    if (name == names[i]) return i;
  return -1;
}

}  // namespace

extern "C" {

int gs_decode_quantity(const char* s, int64_t* value, int64_t* milli_value) {
  int64_t v = 0, mv = 0;
  int rc = quantity_scaled(s, 0, &v);
  if (rc) return rc;
  if ((rc = quantity_scaled(s, 3, &mv))) return rc;
  if (value) *value = v;
  if (milli_value) *milli_value = mv;
  return GS_OK;
}

int gs_decode_cpuset(const char* s, uint64_t out[GS_CPU_WORDS]) {
  if (!s || !out) return GS_EINVAL;
  uint64_t w[GS_CPU_WORDS] = {0, 0, 0, 0};
  auto add = [&](long long c) -> int {
    if (c < 0 || c >= GS_MAX_CPUS) return GS_EUNSUPPORTED;
    w[c >> 6] |= 1ull << (c & 63);
    return GS_OK;
  };
  // strconv.ParseInt(x, 10, 32): optional sign, decimal digits, int32 range
  auto parse_int = [](const std::string& x, long long* v) -> bool {
    if (x.empty()) return false;
    size_t i = (x[0] == '+' || x[0] == '-') ? 1 : 0;
    if (i == x.size()) return false;
    for (size_t j = i; j < x.size(); ++j)
      if (x[j] < '0' || x[j] > '9') return false;
    errno = 0;
    long long r = strtoll(x.c_str(), nullptr, 10);
    if (errno || r < INT32_MIN || r > INT32_MAX) return false;
    *v = r;
    return true;
  };
  const std::string str(s);
  if (!str.empty()) {
    size_t a = 0;
    for (;;) {
      size_t b = str.find(',', a);
      const std::string r = str.substr(a, b == std::string::npos ? std::string::npos : b - a);
      std::vector<std::string> bounds;
      size_t c = 0;
      for (;;) {
        size_t d = r.find('-', c);
        bounds.push_back(r.substr(c, d == std::string::npos ? std::string::npos : d - c));
        if (d == std::string::npos) break;
        c = d + 1;
      }
      long long lo, hi;
      if (bounds.size() == 1) {
        if (!parse_int(bounds[0], &lo)) return GS_EINVAL;
        if (int rc = add(lo)) return rc;
      } else if (bounds.size() == 2) {
        if (!parse_int(bounds[0], &lo) || !parse_int(bounds[1], &hi)) return GS_EINVAL;
        if (hi > 4096) return GS_EINVAL;   // maxAvailableCPUCount (cpuset.go:31)
        for (long long x = lo; x <= hi; ++x)
          if (int rc = add(x)) return rc;
      } else {
        return GS_EINVAL;
      }
      if (b == std::string::npos) break;
      a = b + 1;
    }
  }
  memcpy(out, w, sizeof w);
  return GS_OK;
}

int gs_decode_node_annotations(const gs_kv* kv, uint32_t n, gs_node* node, gs_node_numa* numa) {
  if ((n && !kv) || !node) return GS_EINVAL;
  // node.koordinator.sh/raw-allocatable: GetNodeRawAllocatable; EstimateNode ignores a malformed one
  node->raw_allocatable[0] = node->raw_allocatable[1] = 0;
  node->raw_allocatable_mask = 0;
  if (const char* s = find_kv(kv, n, "node.koordinator.sh/raw-allocatable")) {
    JVal v;
    bool good = parse_json(s, &v) && (v.kind == JVal::OBJ || v.kind == JVal::NUL);
    int64_t vals[2] = {0, 0};
    uint32_t mask = 0;
    if (good && v.kind == JVal::OBJ)
      for (const auto& e : v.obj) {
        int64_t x = 0;
        const bool cpu = e.first == "cpu";
        if (quantity_json(e.second, cpu ? 3 : 0, &x) != GS_OK) { good = false; break; }
        if (cpu) { vals[0] = x; mask |= GS_USAGE_CPU; }
        else if (e.first == "memory") { vals[1] = x; mask |= GS_USAGE_MEMORY; }
      }
    if (good) {
      node->raw_allocatable[0] = vals[0];
      node->raw_allocatable[1] = vals[1];
      node->raw_allocatable_mask = mask;
    }
  }
  // scheduling.koordinator.sh/usage-thresholds: GetCustomUsageThresholds; a malformed one means the args'
  // thresholds (generateUsageThresholdsFilterProfile, helper.go:104-117) = no custom flags
  node->custom_flags = 0;
  node->custom_usage_mask = node->custom_prod_usage_mask = node->custom_agg_usage_mask = 0;
  for (int r = 0; r < 2; ++r)
    node->custom_usage_thresholds[r] = node->custom_prod_usage_thresholds[r] = node->custom_agg_usage_thresholds[r] = 0;
  node->custom_agg_type = GS_AGG_NONE;
  node->custom_agg_duration_ns = 0;
  if (const char* s = find_kv(kv, n, "scheduling.koordinator.sh/usage-thresholds")) {
    JVal v;
    gs_node t = *node;
    bool good = parse_json(s, &v) && (v.kind == JVal::OBJ || v.kind == JVal::NUL);
    if (good && v.kind == JVal::OBJ) {
      good = thresholds_map(v.get("usageThresholds"), t.custom_usage_thresholds, &t.custom_usage_mask) &&
             thresholds_map(v.get("prodUsageThresholds"), t.custom_prod_usage_thresholds, &t.custom_prod_usage_mask);
      const JVal* ag = v.get("aggregatedUsage");
      if (good && ag && ag->kind != JVal::NUL) {
        if (ag->kind != JVal::OBJ) {
          good = false;
        } else {
          t.custom_flags |= GS_NODE_CUSTOM_AGGREGATED;
          good = thresholds_map(ag->get("usageThresholds"), t.custom_agg_usage_thresholds, &t.custom_agg_usage_mask);
          const JVal* ty = ag->get("usageAggregationType");
          if (good && ty && ty->kind != JVal::NUL) {
            if (ty->kind != JVal::STR) good = false;
            else if (int rc = agg_type(ty->text, &t.custom_agg_type)) return rc;   // no device encoding
          }
          const JVal* du = ag->get("usageAggregatedDuration");
          if (good && du && du->kind != JVal::NUL)
            good = du->kind == JVal::STR && parse_duration(du->text, &t.custom_agg_duration_ns);
        }
      }
    }
    if (good) {
      t.custom_flags |= GS_NODE_CUSTOM_THRESHOLDS;
      *node = t;
    }
  }
  // node.koordinator.sh/resource-amplification-ratio: GetNodeResourceAmplificationRatio(cpu); -1 when unset,
  // a parse error fails filterAmplifiedCPUs (plugin.go:345-347)
  if (numa) {
    numa->node_cpu_amplification_ratio = -1;
    numa->node_amplification_invalid = 0;
    if (const char* s = find_kv(kv, n, "node.koordinator.sh/resource-amplification-ratio")) {
      JVal v;
      bool good = parse_json(s, &v) && (v.kind == JVal::OBJ || v.kind == JVal::NUL);
      double cpu = -1;
      if (good && v.kind == JVal::OBJ)
        for (const auto& e : v.obj) {
          double x;
          if (!json_float64(e.second, &x)) { good = false; break; }
          if (e.first == "cpu") cpu = x;
        }
      if (good) numa->node_cpu_amplification_ratio = cpu;
      else numa->node_amplification_invalid = 1;
    }
  }
  return GS_OK;
}

int gs_node_reservation_trim(const gs_kv* kv, uint32_t n, gs_node* node) {
  if ((n && !kv) || !node) return GS_EINVAL;
  NodeRsv r;
  if (!node_reservation(kv, n, &r) || !r.present) return 0;                   // GetNodeReservation error / nil
  if (!(r.apply_policy.empty() || r.apply_policy == "Default")) return 0;     // ReservedCPUsOnly: no trim
  // GetNodeReservationResources (pkg/util/node.go:102-119): the resources, cpu replaced by |reservedCPUs|
  int64_t red[GS_NUM_RES] = {0, 0, 0, 0, 0, 0, 0}, pods = 0;
  bool nonzero = false;
  for (const auto& e : r.resources) {
    const int sl = res_slot(e.first);
    int64_t x = 0;
    const int rc = quantity_json(*e.second, sl == GS_RES_CPU ? 3 : 0, &x);
    if (rc) return rc;   // a negative reserved quantity (it would raise allocatable): refused, see quantity_scaled
    nonzero |= x != 0;
    if (sl >= 0) red[sl] = x;
    else if (e.first == "pods") pods = x;
  }
  if (!r.reserved_cpus.empty()) {
    uint64_t w[GS_CPU_WORDS];
    if (gs_decode_cpuset(r.reserved_cpus.c_str(), w) != GS_OK) return 0;      // cpuset.Parse error: no trim
    int cnt = 0;
    for (int i = 0; i < GS_CPU_WORDS; ++i) cnt += __builtin_popcountll(w[i]);
    // resourceList[cpu] = MustParse(strconv.Itoa(cpus.Size())); the map now always holds cpu
    bool had_nonzero_other = false;
    for (const auto& e : r.resources) {
      if (e.first == "cpu") continue;
      int64_t x = 0;
      (void)quantity_json(*e.second, 0, &x);
      had_nonzero_other |= x != 0;
    }
    red[GS_RES_CPU] = (int64_t)cnt * 1000;
    nonzero = had_nonzero_other || cnt != 0;
  }
  if (!nonzero) return 0;                                                     // quotav1.IsZero
  // SubtractWithNonNegativeResult, then batch-cpu / batch-memory restored (node.go:140-148)
  int changed = 0;
  for (int sl = 0; sl < 7; ++sl) {   // (slot 7 is reserved)
    if (sl == GS_RES_BATCH_CPU || sl == GS_RES_BATCH_MEMORY) continue;
    const int64_t t = node->allocatable[sl] - red[sl] > 0 ? node->allocatable[sl] - red[sl] : 0;
    changed |= t != node->allocatable[sl];
    node->allocatable[sl] = t;
  }
  const int64_t tp = node->allowed_pod_number - pods > 0 ? node->allowed_pod_number - pods : 0;
  changed |= tp != node->allowed_pod_number;
  node->allowed_pod_number = tp;
  return changed;
}

int gs_node_reserved_cpus(const gs_kv* kv, uint32_t n, uint64_t cpus[GS_CPU_WORDS], int32_t* num_reserved_cpus) {
  if ((n && !kv) || !cpus) return GS_EINVAL;
  for (int i = 0; i < GS_CPU_WORDS; ++i) cpus[i] = 0;
  if (num_reserved_cpus) *num_reserved_cpus = 0;
  NodeRsv r;
  if (!node_reservation(kv, n, &r) || !r.present) return GS_OK;
  int32_t num = 0;
  for (const auto& e : r.resources) {
    if (e.first != "cpu") continue;
    int64_t milli = 0;
    if (quantity_json(*e.second, 3, &milli) == GS_OK && milli > 0) num = (int32_t)((milli + 999) / 1000);
  }
  if (!r.reserved_cpus.empty()) num = 0;
  if (num_reserved_cpus) *num_reserved_cpus = num;
  if (r.reserved_cpus.empty()) return GS_OK;
  return gs_decode_cpuset(r.reserved_cpus.c_str(), cpus) == GS_OK ? GS_OK : 1;   // 1: unparsable (no CPUs)
}

int gs_decode_nrt_reserved_cpus(const gs_kv* kv, uint32_t n, uint64_t out[GS_CPU_WORDS]) {
  if ((n && !kv) || !out) return GS_EINVAL;
  uint64_t w[GS_CPU_WORDS] = {0, 0, 0, 0};
  auto unite = [&](const std::string& list) {   // cpuset.Parse; an error is logged by the reference: nothing added
    uint64_t c[GS_CPU_WORDS];
    if (gs_decode_cpuset(list.c_str(), c) != GS_OK) return;
    for (int i = 0; i < GS_CPU_WORDS; ++i) w[i] |= c[i];
  };
  // getPodAllocsCPUSet (topology_options.go:155-171) over GetPodCPUAllocs (numa_aware.go:262-273)
  if (const char* s = find_kv(kv, n, "node.koordinator.sh/pod-cpu-allocs")) {
    JVal v;
    if (parse_json(s, &v) && v.kind == JVal::ARR) {
      bool good = true;
      for (const auto& a : v.arr) good = good && (a.kind == JVal::OBJ || a.kind == JVal::NUL);
      for (size_t i = 0; good && i < v.arr.size(); ++i) {
        const JVal& a = v.arr[i];
        if (a.kind != JVal::OBJ) continue;
        const JVal* mk = a.get("managedByKubelet");
        const JVal* uid = a.get("uid");
        const JVal* cs = a.get("cpuset");
        const bool managed = mk && mk->kind == JVal::BOOL && mk->b;
        if (!managed || !uid || uid->kind != JVal::STR || uid->text.empty() || !cs || cs->kind != JVal::STR ||
            cs->text.empty())
          continue;
        unite(cs->text);
      }
    }
  }
  // kubelet's reserved CPUs (GetKubeletCPUManagerPolicy, numa_aware.go:301-312)
  if (const char* s = find_kv(kv, n, "kubelet.koordinator.sh/cpu-manager-policy")) {
    JVal v;
    if (parse_json(s, &v) && v.kind == JVal::OBJ)
      if (const JVal* rc = v.get("reservedCPUs"))
        if (rc->kind == JVal::STR) unite(rc->text);
  }
  // the node reservation's reservedCPUs (GetReservedCPUs, node_reservation.go:70-90)
  {
    NodeRsv r;
    if (node_reservation(kv, n, &r) && r.present && !r.reserved_cpus.empty()) unite(r.reserved_cpus);
  }
  // an exclusive system-QoS cpuset (GetSystemQOSResource, system_qos.go:35-53)
  if (const char* s = find_kv(kv, n, "node.koordinator.sh/system-qos-resource")) {
    JVal v;
    if (parse_json(s, &v) && v.kind == JVal::OBJ) {
      const JVal* ex = v.get("cpusetExclusive");
      const bool exclusive = !ex || ex->kind == JVal::NUL || (ex->kind == JVal::BOOL && ex->b);
      const JVal* cs = v.get("cpuset");
      if (exclusive && cs && cs->kind == JVal::STR) unite(cs->text);
    }
  }
  memcpy(out, w, sizeof w);
  return GS_OK;
}

int gs_decode_node_labels(const gs_kv* labels, uint32_t n, const char* kubelet_cpu_manager_policy,
                          const char* kubelet_topology_policy, gs_node_numa* numa) {
  if ((n && !labels) || !numa) return GS_EINVAL;
  // GetKubeletCPUManagerPolicy + GetNodeCPUBindPolicy (numa_aware.go:301-325)
  bool full_only_kubelet = false;
  if (kubelet_cpu_manager_policy && *kubelet_cpu_manager_policy) {
    JVal v;
    if (!parse_json(kubelet_cpu_manager_policy, &v) || (v.kind != JVal::OBJ && v.kind != JVal::NUL)) return GS_EINVAL;
    if (v.kind == JVal::OBJ) {
      const JVal* pol = v.get("policy");
      const JVal* opt = v.get("options");
      if ((pol && pol->kind != JVal::STR && pol->kind != JVal::NUL) ||
          (opt && opt->kind != JVal::OBJ && opt->kind != JVal::NUL))
        return GS_EINVAL;
      const JVal* fpo = (opt && opt->kind == JVal::OBJ) ? opt->get("full-pcpus-only") : nullptr;
      if (fpo && fpo->kind != JVal::STR && fpo->kind != JVal::NUL) return GS_EINVAL;
      full_only_kubelet = pol && pol->kind == JVal::STR && pol->text == "static" && fpo && fpo->kind == JVal::STR &&
                          fpo->text == "true";
    }
  }
  const char* bind = find_kv(labels, n, "node.koordinator.sh/cpu-bind-policy");
  if ((bind && strcmp(bind, "FullPCPUsOnly") == 0) || full_only_kubelet)
    numa->node_cpu_bind_policy = GS_NODE_CPU_BIND_FULL_PCPUS_ONLY;
  else if (bind && strcmp(bind, "SpreadByPCPUs") == 0)
    numa->node_cpu_bind_policy = GS_NODE_CPU_BIND_SPREAD_BY_PCPUS;
  else
    numa->node_cpu_bind_policy = GS_NODE_CPU_BIND_NONE;
  // getNUMATopologyPolicy (nodenumaresource/util.go:52-58): the label, else the kubelet topology manager policy
  auto policy = [](const char* s, int32_t* out) -> bool {
    if (!s || !*s) *out = GS_NUMA_POLICY_NONE;
    else if (!strcmp(s, "BestEffort")) *out = GS_NUMA_POLICY_BEST_EFFORT;
    else if (!strcmp(s, "Restricted")) *out = GS_NUMA_POLICY_RESTRICTED;
    else if (!strcmp(s, "SingleNUMANode")) *out = GS_NUMA_POLICY_SINGLE_NUMA_NODE;
    else return false;
    return true;
  };
  int32_t pol = GS_NUMA_POLICY_NONE;
  if (!policy(find_kv(labels, n, "node.koordinator.sh/numa-topology-policy"), &pol)) return GS_EUNSUPPORTED;
  if (pol == GS_NUMA_POLICY_NONE && !policy(kubelet_topology_policy, &pol)) return GS_EUNSUPPORTED;
  numa->numa_topology_policy = pol;
  // GetNUMAAllocateStrategy (util.go:35-41): the label when set, else the args default (UNSET)
  const char* st = find_kv(labels, n, "node.koordinator.sh/numa-allocate-strategy");
  if (!st || !*st) numa->numa_allocate_strategy = GS_NUMA_ALLOC_UNSET;
  else if (!strcmp(st, "MostAllocated")) numa->numa_allocate_strategy = GS_NUMA_ALLOC_MOST_ALLOCATED;
  else if (!strcmp(st, "LeastAllocated")) numa->numa_allocate_strategy = GS_NUMA_ALLOC_LEAST_ALLOCATED;
  else if (!strcmp(st, "DistributeEvenly")) numa->numa_allocate_strategy = GS_NUMA_ALLOC_DISTRIBUTE_EVENLY;
  else return GS_EUNSUPPORTED;
  return GS_OK;
}

int gs_decode_resource_spec(const char* json, gs_pod* pod) {
  if (!pod) return GS_EINVAL;
  pod->required_cpu_bind_policy = pod->preferred_cpu_bind_policy = GS_CPU_BIND_UNSET;
  pod->preferred_cpu_exclusive_policy = GS_CPU_EXCLUSIVE_NONE;
  if (!json) return GS_OK;   // annotation absent: an empty ResourceSpec
  JVal v;
  if (!parse_json(json, &v) || (v.kind != JVal::OBJ && v.kind != JVal::NUL)) return GS_EINVAL;
  if (v.kind == JVal::NUL) return GS_OK;
  auto bind = [](const JVal* x, int32_t* out) -> int {
    if (!x || x->kind == JVal::NUL) return GS_OK;
    if (x->kind != JVal::STR) return GS_EINVAL;
    const std::string& s = x->text;
    if (s.empty()) *out = GS_CPU_BIND_UNSET;
    else if (s == "Default") *out = GS_CPU_BIND_DEFAULT;
    else if (s == "FullPCPUs") *out = GS_CPU_BIND_FULL_PCPUS;
    else if (s == "SpreadByPCPUs") *out = GS_CPU_BIND_SPREAD_BY_PCPUS;
    else if (s == "ConstrainedBurst") *out = GS_CPU_BIND_CONSTRAINED_BURST;
    else return GS_EUNSUPPORTED;
    return GS_OK;
  };
  int32_t req = GS_CPU_BIND_UNSET, pref = GS_CPU_BIND_UNSET, ex = GS_CPU_EXCLUSIVE_NONE;
  if (int rc = bind(v.get("requiredCPUBindPolicy"), &req)) return rc;
  if (int rc = bind(v.get("preferredCPUBindPolicy"), &pref)) return rc;
  if (const JVal* x = v.get("preferredCPUExclusivePolicy"); x && x->kind != JVal::NUL) {
    if (x->kind != JVal::STR) return GS_EINVAL;
    if (x->text.empty() || x->text == "None") ex = GS_CPU_EXCLUSIVE_NONE;
    else if (x->text == "PCPULevel") ex = GS_CPU_EXCLUSIVE_PCPU_LEVEL;
    else if (x->text == "NUMANodeLevel") ex = GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL;
    else return GS_EUNSUPPORTED;
  }
  pod->required_cpu_bind_policy = req;
  pod->preferred_cpu_bind_policy = pref;
  pod->preferred_cpu_exclusive_policy = ex;
  return GS_OK;
}

int gs_decode_cpu_topology(const char* json, gs_cpu_topology* out) {
  if (!out) return GS_EINVAL;
  memset(out, 0, sizeof *out);
  if (!json) return GS_OK;   // annotation absent: an empty CPUTopology
  JVal v;
  if (!parse_json(json, &v) || (v.kind != JVal::OBJ && v.kind != JVal::NUL)) return GS_EINVAL;
  const JVal* d = v.kind == JVal::OBJ ? v.get("detail") : nullptr;
  if (!d || d->kind == JVal::NUL) return GS_OK;
  if (d->kind != JVal::ARR) return GS_EINVAL;
  // CPUTopologyBuilder.AddCPUInfo keys CPUDetails by id; the device tables need ids 0..num_cpus-1
  std::vector<int> seen(GS_MAX_CPUS, 0);
  int maxid = -1;
  for (const JVal& c : d->arr) {
    if (c.kind != JVal::OBJ) return GS_EINVAL;
    int32_t id = 0, core = 0, socket = 0, node = 0;
    const JVal* f;
    if ((f = c.get("id")) && f->kind != JVal::NUL && !json_int32(*f, &id)) return GS_EINVAL;
    if ((f = c.get("core")) && f->kind != JVal::NUL && !json_int32(*f, &core)) return GS_EINVAL;
    if ((f = c.get("socket")) && f->kind != JVal::NUL && !json_int32(*f, &socket)) return GS_EINVAL;
    if ((f = c.get("node")) && f->kind != JVal::NUL && !json_int32(*f, &node)) return GS_EINVAL;
    if (id < 0 || id >= GS_MAX_CPUS || socket < 0 || socket > 255 || node < 0 || node > 255 || core < 0 ||
        core > 0xFFFF)
      return GS_EUNSUPPORTED;
    seen[id] = 1;
    out->core_id[id] = (socket << 16) | core;   // cpu_topology.go:45
    out->socket_id[id] = (uint8_t)socket;
    out->node_id[id] = (uint8_t)node;
    if (id > maxid) maxid = id;
  }
  for (int i = 0; i <= maxid; ++i)
    if (!seen[i]) return GS_EUNSUPPORTED;   // a hole in the CPU ids
  out->num_cpus = maxid + 1;
  return GS_OK;
}

}  // extern "C"
