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
//
// columnize_batch() decodes many requests on `threads` worker threads against
// a read-only view of the dictionaries, then commits them in request order; a
// request that meets anything new (resource, service, series) or fails is
// redone by the calling thread at its place in that order, so the columns,
// ids and reports are the ones request-at-a-time columnize() would give.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <utility>
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
  bool test_batched = false;                // tests only: the batched span path whenever it applies
  unsigned threads = 1;                     // columnize_batch worker threads (caller included)
  // aggregation_cardinality_limit: past this many span series in a resource,
  // new keys share the resource's overflow series (0 = unlimited)
  uint32_t card_limit = 0;
  // exemplars.enabled / max_per_data_point: the first `exemplars_max` spans
  // of every series per export interval are reported (their offsets)
  bool exemplars = false;
  uint32_t exemplars_max = 5;
  // events.enabled / events.dimensions: one record per span event, keyed by
  // the span's key and the event dimensions
  bool events = false;
  std::vector<Dim> event_dims;
};

struct NewSeries {
  uint64_t sid, res_hash;
  uint32_t span_off, span_len;  // the Span message inside the request bytes
  int64_t res_off = -1;         // its Resource message (-1: absent); the host keys
  uint32_t res_len = 0;         // dimensions with this resource's own attributes
};

// An exemplar candidate / a new event series: the span (offsets in the
// request bytes) and, for events, which of its events
struct SpanRef {
  uint64_t sid;
  uint32_t span_off, span_len;
  // exemplars: the span's fields an exemplar carries, when its trace id is 16
  // bytes and its span id 8 (ids_ok; else the host decodes the span itself)
  bool ids_ok = false;
  uint8_t ids[24] = {};  // trace id, then span id
  uint64_t start = 0, end = 0;
};
struct NewEventSeries {
  uint64_t sid, res_hash;
  uint32_t span_off, span_len, event;
  int64_t res_off = -1;  // as NewSeries
  uint32_t res_len = 0;
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
  std::vector<SpanRef> exemplars;                 // accepted exemplar spans, in arrival order
  std::vector<NewEventSeries> new_event_series;   // event series this request made
  uint64_t event_records = 0;                     // event records appended to the columns
};

struct BatchResult {
  std::vector<Result> results;  // one per request taken, in order
  size_t done = 0;              // requests taken: all, or up to and including the first fallback
  // wall time of the three phases (threaded calls): the parallel decode, the
  // in-order commit (exclusive redos, exemplar acceptance) and the parallel
  // copy into the column buffer
  uint64_t ns_decode = 0, ns_commit = 0, ns_place = 0;
};

// Column storage.  The columnizer's output buffer asks for page-locked host
// memory through hooks the addon installs (libspanagg's sa_host_alloc), so
// sa_ingest DMAs it to HBM without packing a staging copy on the calling
// thread; worker scratch and any failed pinned allocation use the heap.
// Every block carries a 64-B header naming its kind, for deallocation.
using HostAllocFn = void *(*)(size_t);
using HostFreeFn = void (*)(void *);
void set_host_allocator(HostAllocFn a, HostFreeFn f);
void *col_alloc(size_t bytes, bool pinned);
void col_free(void *p);
template <class T>
struct ColAlloc {
  using value_type = T;
  bool pinned = false;
  ColAlloc() = default;
  explicit ColAlloc(bool p) : pinned(p) {}
  template <class U>
  ColAlloc(const ColAlloc<U> &o) : pinned(o.pinned) {}
  T *allocate(size_t n) { return static_cast<T *>(col_alloc(n * sizeof(T), pinned)); }
  void deallocate(T *p, size_t) { col_free(p); }
  bool operator==(const ColAlloc &o) const { return pinned == o.pinned; }
  bool operator!=(const ColAlloc &o) const { return pinned != o.pinned; }
};
template <class T>
using ColVec = std::vector<T, ColAlloc<T>>;

// SoA v1 columns under construction.  The six arrays share one capacity
// (their vector size) and one fill count n, so appending a span is one bound
// check and six stores.
struct Cols {
  ColVec<uint64_t> key, start, end, w0, w1;
  ColVec<uint32_t> meta;
  size_t n = 0;
  uint64_t max_end = 0;
  Cols() = default;
  explicit Cols(bool pinned)
      : key(ColAlloc<uint64_t>(pinned)), start(ColAlloc<uint64_t>(pinned)), end(ColAlloc<uint64_t>(pinned)),
        w0(ColAlloc<uint64_t>(pinned)), w1(ColAlloc<uint64_t>(pinned)), meta(ColAlloc<uint32_t>(pinned)) {}
  size_t size() const { return n; }
  void reserve(size_t cap);  // capacity for at least cap spans (contents kept)
  void push(uint64_t k, uint64_t s, uint64_t e, uint64_t a, uint64_t b, uint32_t m) {
    if (n == key.size()) reserve(n + 1);
    key[n] = k, start[n] = s, end[n] = e, w0[n] = a, w1[n] = b, meta[n] = m;
    ++n;
  }
  void truncate(size_t m) { n = m; }
  void clear() { n = 0, max_end = 0; }
};

// A zeroed array of trivially copyable T; from 2 MiB up 2 MiB-aligned and
// madvise(MADV_HUGEPAGE)d: a high-cardinality signature table is far larger
// than the TLB's 4 KiB-page reach, and a page walk on every lookup cost more
// than the lookup's one cache miss.
template <typename T>
class BigArray {
 public:
  BigArray() = default;
  BigArray(const BigArray &) = delete;
  BigArray &operator=(const BigArray &) = delete;
  ~BigArray() { std::free(p_); }
  void assign_zero(size_t n);  // n elements, all zero bytes (the old contents are dropped)
  void swap(BigArray &o) { std::swap(p_, o.p_), std::swap(n_, o.n_); }
  void clear() { std::free(p_), p_ = nullptr, n_ = 0; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T &operator[](size_t i) { return p_[i]; }
  const T &operator[](size_t i) const { return p_[i]; }
  const T *begin() const { return p_; }
  const T *end() const { return p_ + n_; }

 private:
  T *p_ = nullptr;
  size_t n_ = 0;
};

// (resource hash, service id, raw span name, kind, status code) -> series id,
// for keys without dimensions: a span of a known series skips UTF-8
// validation, the rename rules and building its key string
class SigCache {
 public:
  static uint64_t hash(uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind, int32_t code);
  struct Entry;
  struct Rec;
  // the record of the signature, or null; rec_entry gives its Entry (the
  // rarely read fields: exemplar mark, event key)
  const Rec *find(uint64_t h, uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind, int32_t code) const;
  Entry &rec_entry(const Rec *r) { return entries_[r->idx]; }
  // the signature's home record and the next (linear probing: a hit at load
  // <= 1/2 is past its home one time in ~4)
  void prefetch(uint64_t h) const {
    if (recs_.empty()) return;
    const size_t mask = recs_.size() - 1;
    __builtin_prefetch(&recs_[h & mask]);
    __builtin_prefetch(&recs_[(h + 1) & mask]);
  }
  const Entry &rec_entry(const Rec *r) const { return entries_[r->idx]; }
  // key: the span's key string, kept for events.enabled (its spans' event
  // keys extend it), empty otherwise.  A kind or code outside int16 is never
  // cached (find misses, the caller keys the span the long way).
  void insert(uint64_t h, uint64_t rhash, uint32_t svc, std::string_view name, int32_t kind, int32_t code,
              uint64_t sid, const std::string &key);
  static bool cacheable(int32_t kind, int32_t code) {
    return kind == (int16_t)kind && code == (int16_t)code;
  }
  void clear() { recs_.clear(), entries_.clear(), names_.clear(), fresh_.clear(); }
  size_t size() const { return entries_.size(); }
  uint64_t gen = 0;  // the dictionary generation the entries belong to
  // entries inserted since the last take_fresh (a worker's, merged into the
  // shared cache after each batch)
  template <typename F> void take_fresh(F &&f) {
    for (uint32_t i : fresh_) {
      const Entry &e = entries_[i];
      f(e, std::string_view(names_.data() + e.name_off, e.name_len));
    }
    fresh_.clear();
  }
  void drop_fresh() { fresh_.clear(); }

  struct Entry {
    uint64_t h = 0, rhash = 0, sid = 0;
    uint64_t ex_full = 0;  // the exemplar interval (Columnizer::ex_gen_) in which the series was seen full
    uint32_t svc = 0;
    int32_t kind = 0, code = 0;
    uint32_t name_off = 0, name_len = 0;  // the signature name in names_
    std::string key;                      // events.enabled: the span key string (see insert)
  };
  // One cache line holds everything a lookup compares and its answer: the
  // full hash, the series id, the signature's fields and, for a name of at
  // most kInline bytes, the name itself (a longer one is compared in names_,
  // which holds every name).  A high-cardinality stream's table is far larger
  // than the CPU caches, so a hit costs one memory access (two for a longer
  // name) instead of the three of a slot array, an entry array and a name
  // arena.
  static constexpr uint32_t kInline = 20;
  struct alignas(64) Rec {
    uint64_t h;  // 0: free
    uint64_t sid, rhash;
    uint32_t svc;
    int16_t kind, code;
    uint32_t name_len, name_off, idx;  // the name in names_, the Entry
    char name[kInline];
  };
  static_assert(sizeof(Rec) == 64, "one cache line");

 private:
  BigArray<Rec> recs_;  // open addressing, linear probing, load <= 1/2
  std::vector<Entry> entries_;
  std::string names_;
  std::vector<uint32_t> fresh_;
};

class Columnizer {
 public:
  explicit Columnizer(Options o);
  ~Columnizer();

  // Appends the request's spans to the column buffer (all or nothing).
  Result columnize(const uint8_t *buf, size_t len);
  // Many requests (see the header comment); stops after the first fallback,
  // which the caller handles before passing the rest again.
  BatchResult columnize_batch(const uint8_t *const *bufs, const size_t *lens, size_t n);

  uint32_t service_id(const std::string &name, bool *is_new);
  void forget_resource(uint64_t hash) { res_keys_.erase(hash), nspan_.erase(hash), ++gen_; }
  // the host interned (resource, key) as `sid` (a series its JavaScript path saw first)
  void learn(uint64_t rhash, const std::string &key, uint64_t sid);
  // the host's id for a series this columnizer reported as `from` is `to`:
  // buffered spans and the dictionary follow (the host's dictionary decides)
  void remap(uint64_t from, uint64_t to);
  void clear_buffer() { buf_.clear(); }
  // The buffer just handed to the engine's asynchronous DMA (sa_ingest_async)
  // becomes the spare and columnizing continues into the other one; the
  // engine returns from its next sa_ingest_async only once the spare has been
  // read, so the two alternate.
  void swap_buffers() {
    std::swap(buf_, spare_);
    buf_.clear();
  }
  // a new export interval: every series may take exemplars again
  void reset_exemplars() { ex_count_.clear(), ++ex_gen_; }

  size_t buffered() const { return buf_.size(); }
  uint64_t max_end() const { return buf_.max_end; }
  const uint64_t *key() const { return buf_.key.data(); }
  const uint64_t *start() const { return buf_.start.data(); }
  const uint64_t *end() const { return buf_.end.data(); }
  const uint64_t *w0() const { return buf_.w0.data(); }
  const uint64_t *w1() const { return buf_.w1.data(); }
  const uint32_t *meta() const { return buf_.meta.data(); }

 private:
  struct Worker;  // per-thread scratch, columns and signature cache
  struct Undo;    // dictionary entries made by one exclusive call
  struct Pool;
  Result columnize_into(const uint8_t *buf, size_t len, Cols &out);
  // cache: the thread's own signature cache; l2: the shared one (read only
  // while workers decode; filled from the workers' new entries between batches)
  template <bool kShared>
  bool run(const uint8_t *buf, size_t len, Worker &w, Cols &out, SigCache &cache, const SigCache *l2, Result &res,
           Undo *undo);

  Options opt_;
  Cols buf_{true}, excl_;  // buf_: page-locked when possible; excl_: a batch's exclusively redone requests
  Cols spare_{true};       // the other page-locked buffer (swap_buffers)
  SigCache cache_;
  SigCache shared_;  // every thread's signatures, second level (see run)
  uint64_t gen_ = 0;  // bumped whenever an existing dictionary entry may change
  std::unique_ptr<Worker> main_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::unique_ptr<Pool> pool_;
  std::unordered_map<std::string, uint32_t> services_;
  std::unordered_map<uint64_t, std::unordered_map<std::string, uint64_t>> res_keys_;
  // every id handed out -> its (resource, key): an id held by another series
  // is re-salted (seed + 1) instead of shared; kept after a resource is
  // forgotten, so the same series gets the same id when it comes back
  std::unordered_map<uint64_t, std::pair<uint64_t, std::string>> owner_;
  // span series per resource (aggregation_cardinality_limit)
  std::unordered_map<uint64_t, uint32_t> nspan_;
  // exemplars taken per series this export interval (written in request order)
  std::unordered_map<uint64_t, uint32_t> ex_count_;
  uint64_t ex_gen_ = 1;  // the exemplar interval, for SigCache::Entry::ex_full
  // keeps the request's exemplar candidates that the interval still wants
  void accept_exemplars(Result &r);
};

// exposed for tests of the building blocks
uint64_t xxh64(const void *data, size_t len, uint64_t seed);
std::string format_float(double v);  // Go strconv.FormatFloat(v, 'f', -1, 64)
std::string apply_rules(const std::vector<Rule> &rules, std::string name);

}  // namespace otlpcol
