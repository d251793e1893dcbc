'use strict';
/**
 * Host-side rate of the Node path: OTLP/protobuf request bytes -> decode ->
 * transform rules -> keying -> SoA columns -> addon.ingest.  SURVEY.md 8(d)
 * asks for the OTLP decode+aggregate rate from protobuf bytes.
 *
 *   node test/host_rate.js [spans] [--gpu] [--threads T] [--batch B] [--exemplars] [--events] [--highcard]
 *                          [--dump FILE]
 *
 * --threads T --batch B: requests go through consumeTracesBatch B at a time
 * (what the pipeline's queue does under load), decoded on T columnizer
 * threads (the JavaScript thread is one of them); default T=1, one request at a time.
 * Without --gpu the addon's ingest is a no-op stub (host work only); with
 * --gpu the real addon ingests (host memory -> HBM -> kernel) and the result
 * is checked for span count.  --exemplars: exemplars.enabled (5 per data
 * point); --events: events.enabled on exception.type, with one span in 16
 * carrying an exception event.  --highcard: BASELINE config 4's vocabulary --
 * 500 pods (resource attribute k8s.pod.name) x 2,000 routes (span attribute
 * http.route, a configured dimension) = 1 M series over a binned engine
 * table; the warm-up is a whole pass over the requests, so the timed pass
 * sees every series known, as a long-running collector does.  Prints one
 * JSON line.
 */
const path = require('path');
const lib = path.join(__dirname, '..', 'lib');
const otlp = require(path.join(lib, 'otlp'));
const { TracesToMetricsPipeline } = require(path.join(lib, 'pipeline'));
const { NativeColumnizerFakeAddon } = require('./fake_addon');

const n = parseInt(process.argv[2] || '200000', 10);
const gpu = process.argv.includes('--gpu');
const jsOnly = process.argv.includes('--js');  // force the JavaScript columnizer
const argOf = (k, d) => { const i = process.argv.indexOf(k); return i > 0 ? parseInt(process.argv[i + 1], 10) : d; };
const threads = argOf('--threads', 1), batch = argOf('--batch', 0);
const exemplars = process.argv.includes('--exemplars'), events = process.argv.includes('--events');
const highcard = process.argv.includes('--highcard');
const PER_REQUEST = 512;  // an SDK batch span processor's default export batch
const SERVICES = 20, NAMES = 25, PODS = 500, ROUTES = 2000;

function makeRequests() {
  // mulberry32: successive draws independent enough that --highcard's pod x
  // route pairs really span the 1 M combinations (the LCG used before had
  // correlated consecutive outputs: ~112 k distinct series)
  let seed = 42;
  const rnd = () => {
    seed = (seed + 0x6D2B79F5) | 0;
    let t = Math.imul(seed ^ (seed >>> 15), 1 | seed);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
  const reqs = [];
  const T0 = 1700000000000000000n;
  for (let done = 0; done < n; done += PER_REQUEST) {
    const pod = highcard ? Math.floor(rnd() * PODS) : 0;
    const svc = highcard ? pod % SERVICES : Math.floor(rnd() * SERVICES);
    const spans = [];
    for (let i = 0; i < Math.min(PER_REQUEST, n - done); i++) {
      const route = highcard ? Math.floor(rnd() * ROUTES) : 0;
      const name = highcard ? route % NAMES : Math.floor(rnd() * NAMES);
      const start = T0 + BigInt(Math.floor(rnd() * 6e10));
      const tid = new Uint8Array(16);
      for (let k = 0; k < 16; k++) tid[k] = Math.floor(rnd() * 256);
      spans.push({ traceId: tid, spanId: tid.subarray(0, 8), name: name % 5 === 0 ? `GET /api/products/${name}?x=1` : `op-${name}`,
        kind: 2, startTimeUnixNano: start, endTimeUnixNano: start + BigInt(Math.floor(rnd() * 2e7)),
        attributes: highcard ? [{ key: 'http.method', value: { type: 'string', value: 'GET' } },
          { key: 'http.route', value: { type: 'string', value: `/api/r${route}` } }]
          : [{ key: 'http.method', value: { type: 'string', value: 'GET' } }],
        status: { code: rnd() < 0.02 ? 2 : 0, message: '' },
        events: events && (i & 15) === 0 ? [{ timeUnixNano: start, name: 'exception',
          attributes: [{ key: 'exception.type', value: { type: 'string', value: `E${name % 3}` } }] }] : [] });
    }
    const resAttrs = [{ key: 'service.name', value: { type: 'string', value: `svc-${svc}` } },
      { key: 'telemetry.sdk.language', value: { type: 'string', value: 'go' } }];
    if (highcard) resAttrs.push({ key: 'k8s.pod.name', value: { type: 'string', value: `pod-${pod}` } });
    reqs.push(otlp.encodeTraces({ resourceSpans: [{ resource: { attributes: resAttrs },
      scopeSpans: [{ scope: { name: 'bench' }, spans }] }] }));
  }
  return reqs;
}

const reqs = makeRequests();
const bytes = reqs.reduce((a, b) => a + b.length, 0);
// --dump FILE: write the requests (u32 little-endian length + bytes each) for
// tools/colbench (the columnizer alone, profiled natively) and exit
const dumpAt = process.argv.indexOf('--dump');
if (dumpAt > 0) {
  const fs = require('fs');
  const parts = [];
  for (const r of reqs) {
    const len = Buffer.alloc(4);
    len.writeUInt32LE(r.length, 0);
    parts.push(len, Buffer.from(r.buffer, r.byteOffset, r.length));
  }
  fs.writeFileSync(process.argv[dumpAt + 1], Buffer.concat(parts));
  console.log(JSON.stringify({ dumped: reqs.length, spans: n, otlp_bytes: bytes }));
  process.exit(0);
}
let addon;
if (gpu) {
  addon = require(path.join(lib, 'addon')).load();
} else {
  addon = new NativeColumnizerFakeAddon();  // the real columnizer, no engine
  addon.ingest = () => {};                  // host work only
  addon.columnizerIngest = (c) => addon.real.columnizerTake(c).keyHash.length;
}
// time spent inside the addon's batch columnizer and its ingest (the rest of
// the timed region is the JavaScript thread's own work)
const spent = { columnize: 0n, ingest: 0n, sync: 0n, apply: 0n };
const timed = (obj, fn, k) => {
  const orig = obj[fn].bind(obj);
  obj[fn] = (...a) => {
    const t = process.hrtime.bigint();
    try { return orig(...a); } finally { spent[k] += process.hrtime.bigint() - t; }
  };
};
for (const [fn, k] of [['columnizeBatch', 'columnize'], ['columnizerIngest', 'ingest'], ['sync', 'sync']]) {
  if (addon[fn]) timed(addon, fn, k);
}
// columnize_batch's own phases (decode / commit / place), summed over the calls
const phases = [0, 0, 0, 0, 0];
{
  const cb = addon.columnizeBatch;
  addon.columnizeBatch = (...a) => {
    const r = cb(...a);
    if (r && r.phaseNs) for (let i = 0; i < r.phaseNs.length; i++) phases[i] += r.phaseNs[i];
    return r;
  };
}
const p = new TracesToMetricsPipeline({ addon, receiver: false, exporter: false, memoryLimiter: false,
  native: !jsOnly, spanmetrics: Object.assign({ n_services: 64, columnizer_threads: threads },
    highcard ? { dimensions: [{ name: 'http.route' }], key_capacity: 1200000 } : {},
    exemplars ? { exemplars: { enabled: true, max_per_data_point: 5 } } : {},
    events ? { events: { enabled: true, dimensions: [{ name: 'exception.type' }] } } : {}) });
timed(p.connector, '_applyNative', 'apply');  // the host bookkeeping of the non-plain results
const consumeAll = (list) => {
  if (!batch) { for (const r of list) p.consumeTraces(r); return; }
  for (let i = 0; i < list.length; i += batch) {
    const errs = p.connector.consumeTracesBatch(list.slice(i, i + batch));
    if (errs.some(Boolean)) throw errs.find(Boolean);
  }
};
// warm-up on a tenth of the requests (JIT), then time the whole set
// (--highcard: a whole pass, so every series is known when the timing starts)
const warm = highcard ? reqs : reqs.slice(0, Math.max(1, Math.floor(reqs.length / 10)));
consumeAll(warm);
const warmSpans = BigInt(Math.min(n, warm.length * PER_REQUEST));
p.connector.exportMetrics();
spent.columnize = spent.ingest = spent.sync = spent.apply = 0n;
phases.fill(0);
const t0 = process.hrtime.bigint();
consumeAll(reqs);
p.connector._drain();
if (gpu) addon.sync(p.connector.handle);
const secs = Number(process.hrtime.bigint() - t0) / 1e9;
const out = p.connector.exportMetrics();
let calls = 0n;
let nEx = 0;
for (const rm of out.resourceMetrics) {
  for (const m of rm.scopeMetrics[0].metrics) {
    if (m.name === 'traces.span.metrics.calls') for (const dp of m.sum.dataPoints) calls += dp.asInt;
    if (m.histogram) for (const dp of m.histogram.dataPoints) nEx += (dp.exemplars || []).length;
  }
}
const st = p.connector.stats();
const native = st.nativeRequests > 0 && st.jsRequests === 0;
p.shutdown();
console.log(JSON.stringify({ spans: n, requests: reqs.length, otlp_bytes: bytes, seconds: secs,
  spans_per_s: n / secs, mb_per_s: bytes / secs / 1e6, cores: threads, batch, gpu, highcard,
  series: st.series,
  seconds_in: { columnize_batch: Number(spent.columnize) / 1e9, ingest: Number(spent.ingest) / 1e9,
    sync: Number(spent.sync) / 1e9, apply_native: Number(spent.apply) / 1e9,
    columnize_phases: { decode: phases[0] / 1e9, commit: phases[1] / 1e9, place: phases[2] / 1e9,
      napi_args: phases[3] / 1e9, napi_results: phases[4] / 1e9 } },
  columnizer: native ? 'native (binding/otlp_columnizer.cc)' : 'javascript',
  exemplars: exemplars ? nEx : undefined, event_records: events ? Number(st.eventRecords) : undefined,
  calls_check: gpu ? calls === BigInt(n) + warmSpans : null,  // cumulative: warm-up + timed
  path: 'OTLP protobuf decode + transform + keying + SoA columnize' + (gpu ? ' + sa_ingest (H2D + kernel)' : ' (engine ingest stubbed)') }));
