// otlp_columnizer.h -- native OTLP/protobuf -> SoA v1 columnizer for the
// Node host.  It does in one pass over the request bytes
// what lib/otlp.js + lib/transform.js + lib/keys.js + the connector's
// consumeTraces do in JavaScript for the default option set, and must agree
// with them byte for byte:
//
//   - skip resources without service.name (A1); a non-string service.name keys as ""
//   - resource identity = keys.js resourceHash (xxh64 over sorted
//     key \0 AsString(value) \0 type-tag \1, last duplicate wins), optionally
//     over resource_metrics_key_attributes only
//   - span name through the transform rules (Go regexp `\?.*` strip, whole-value glob)
//   - key = svc \0 name \0 SpanKindStr \0 StatusCodeStr [\0 dim]* (exclusions,
//     missing dims skipped, defaults), series id = xxh64(resHash LE || key)
//   - meta = service id | kind << 16 | status << 19 (clamped as the JS path does)
//
// Anything outside that subset (array / kvlist values where a string form is
// needed) makes columnize() report a fallback and roll back, and the host
// handles that request in JavaScript.  Decoding errors roll back too.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace otlpcol {

struct Rule {
  enum Kind { kStripQuery, kGlob } kind;
  std::string pattern, replacement;  // kGlob: `*` any run, `?` one code point
  // kGlob, derived by prepare(): the pattern's code points and its literal prefix
  std::vector<uint32_t> cps;
  std::string prefix;
  void prepare();
};

struct Dim {
  std::string name;
  bool has_default = false;
  std::string def;
};

struct Options {
  std::vector<Dim> dims;
  bool ex_service = false, ex_name = false, ex_kind = false, ex_status = false;
  std::vector<Rule> rules;
  std::vector<std::string> key_attributes;  // resource_metrics_key_attributes (empty = all)
  bool test_collide_seed0 = false;          // tests only: every seed-0 series id is 42
};

struct NewSeries {
  uint64_t sid, res_hash;
  uint32_t span_off, span_len;  // the Span message inside the request bytes
};

struct NewResource {
  uint64_t hash;
  int64_t off;  // the Resource message (-1: absent -> no attributes)
  uint32_t len;
};

struct Result {
  enum Status { kOk, kFallback, kError } status = kOk;
  std::string error;
  uint64_t spans = 0;
  std::vector<NewResource> new_resources;
  std::vector<NewSeries> new_series;
  std::vector<uint64_t> resources;  // resource hash of every ResourceSpans that contributed
  std::vector<std::pair<std::string, uint32_t>> new_services;
};

class Columnizer {
 public:
  explicit Columnizer(Options o) : opt_(std::move(o)) {}

  // Appends the request's spans to the column buffer (all or nothing).
  Result columnize(const uint8_t *buf, size_t len);

  uint32_t service_id(const std::string &name, bool *is_new);
  void forget_resource(uint64_t hash) { res_keys_.erase(hash); }
  // the host interned (resource, key) as `sid` (a series its JavaScript path saw first)
  void learn(uint64_t rhash, const std::string &key, uint64_t sid);
  // the host's id for a series this columnizer reported as `from` is `to`:
  // buffered spans and the dictionary follow (the host's dictionary decides)
  void remap(uint64_t from, uint64_t to);
  void clear_buffer() {
    key_.clear(); start_.clear(); end_.clear(); w0_.clear(); w1_.clear(); meta_.clear();
    max_end_ = 0;
  }

  size_t buffered() const { return key_.size(); }
  uint64_t max_end() const { return max_end_; }
  const uint64_t *key() const { return key_.data(); }
  const uint64_t *start() const { return start_.data(); }
  const uint64_t *end() const { return end_.data(); }
  const uint64_t *w0() const { return w0_.data(); }
  const uint64_t *w1() const { return w1_.data(); }
  const uint32_t *meta() const { return meta_.data(); }

 private:
  Options opt_;
  std::vector<uint64_t> key_, start_, end_, w0_, w1_;
  std::vector<uint32_t> meta_;
  uint64_t max_end_ = 0;
  std::unordered_map<std::string, uint32_t> services_;
  std::unordered_map<uint64_t, std::unordered_map<std::string, uint64_t>> res_keys_;
  // every id handed out -> its (resource, key): an id held by another series
  // is re-salted (seed + 1) instead of shared; kept after a resource is
  // forgotten, so the same series gets the same id when it comes back
  std::unordered_map<uint64_t, std::pair<uint64_t, std::string>> owner_;
};

// exposed for tests of the building blocks
uint64_t xxh64(const void *data, size_t len, uint64_t seed);
std::string format_float(double v);  // Go strconv.FormatFloat(v, 'f', -1, 64)
std::string apply_rules(const std::vector<Rule> &rules, std::string name);

}  // namespace otlpcol
