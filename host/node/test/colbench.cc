// colbench -- the native OTLP columnizer (binding/otlp_columnizer.cc) alone,
// over OTLP requests dumped by `node test/host_rate.js N [--events] --dump F`:
// decode + transform rules + keying + SoA columns, in batches through
// columnize_batch on T threads (the addon's consumeTracesBatch path without
// N-API or the engine).  Prints one JSON line with the rate and the time in
// each columnize_batch phase.  A profiling tool, not part of the addon.
//
//   colbench FILE [--threads T] [--batch B] [--reps R] [--exemplars] [--events] [--dim NAME]...
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "../binding/otlp_columnizer.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: colbench FILE [--threads T] [--batch B] [--reps R] [--exemplars] [--events] [--dim NAME]...\n");
    return 2;
  }
  unsigned threads = 1, batch = 128, reps = 5;
  bool exemplars = false, events = false;
  std::vector<std::string> dims;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--threads" && i + 1 < argc) threads = (unsigned)std::atoi(argv[++i]);
    else if (a == "--batch" && i + 1 < argc) batch = (unsigned)std::atoi(argv[++i]);
    else if (a == "--reps" && i + 1 < argc) reps = (unsigned)std::atoi(argv[++i]);
    else if (a == "--exemplars") exemplars = true;
    else if (a == "--events") events = true;
    else if (a == "--dim" && i + 1 < argc) dims.push_back(argv[++i]);  // a dimension (no default)
  }
  std::ifstream f(argv[1], std::ios::binary);
  const std::vector<uint8_t> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<const uint8_t *> bufs;
  std::vector<size_t> lens;
  for (size_t o = 0; o + 4 <= raw.size();) {
    uint32_t n;
    std::memcpy(&n, raw.data() + o, 4);
    bufs.push_back(raw.data() + o + 4);
    lens.push_back(n);
    o += 4 + n;
  }
  otlpcol::Options o;
  o.threads = threads;
  // the demo's two transform statements (otelcol-config.yml:111-113)
  o.rules.push_back({otlpcol::Rule::kStripQuery, "", "", {}, ""});
  o.rules.push_back({otlpcol::Rule::kGlob, "GET /api/products/*", "GET /api/products/{productId}", {}, ""});
  for (auto &r : o.rules) r.prepare();
  o.exemplars = exemplars;
  o.events = events;
  if (events) o.event_dims.push_back({"exception.type", false, ""});
  for (const std::string &d : dims) o.dims.push_back({d, false, ""});
  otlpcol::Columnizer col(o);
  using clk = std::chrono::steady_clock;
  double best = 1e30, dec = 0, com = 0, pla = 0;
  uint64_t spans = 0;
  for (unsigned r = 0; r <= reps; ++r) {  // rep 0 warms the dictionaries and caches
    col.clear_buffer();
    col.reset_exemplars();
    uint64_t s = 0, nd = 0, nc = 0, np = 0;
    const auto t0 = clk::now();
    for (size_t i = 0; i < bufs.size(); i += batch) {
      const size_t m = std::min<size_t>(batch, bufs.size() - i);
      otlpcol::BatchResult br = col.columnize_batch(bufs.data() + i, lens.data() + i, m);
      for (auto &x : br.results) s += x.spans;
      nd += br.ns_decode, nc += br.ns_commit, np += br.ns_place;
      col.clear_buffer();
    }
    const double sec = std::chrono::duration<double>(clk::now() - t0).count();
    if (r > 0 && sec < best) best = sec, dec = nd * 1e-9, com = nc * 1e-9, pla = np * 1e-9, spans = s;
  }
  std::printf("{\"spans\": %llu, \"requests\": %zu, \"threads\": %u, \"batch\": %u, \"exemplars\": %s, \"events\": %s, "
              "\"seconds\": %.6f, \"spans_per_s\": %.4g, \"mb_per_s\": %.1f, "
              "\"seconds_in\": {\"decode\": %.6f, \"commit\": %.6f, \"place\": %.6f}}\n",
              (unsigned long long)spans, bufs.size(), threads, batch, exemplars ? "true" : "false",
              events ? "true" : "false", best, spans / best, raw.size() / best / 1e6, dec, com, pla);
  return 0;
}
