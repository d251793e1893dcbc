'use strict';
/**
 * End-to-end run of the Node host on the real addon (GPU): OTLP request bytes
 * -> decode -> demo transform rules -> SpanMetricsConnector (libspanagg on the
 * GPU) -> exportMetrics -> OTLP metrics bytes.  Driven by
 * tests/test_node_host.py, which checks every stage against independent
 * Python code (protobuf, keys.py) and the C oracle.
 *
 * stdin:  {"requests": [b64...], "config": {...}, "exports_after": [i...]}
 * stdout: {"columns": {col: b64}, "flushes": [...], "metrics": [b64...],
 *          "windows": [{window_id, hll, cms}], "stats": {...}}
 */
const path = require('path');
const lib = path.join(__dirname, '..', 'lib');
const addonLoader = require(path.join(lib, 'addon'));
const otlp = require(path.join(lib, 'otlp'));
const { DEMO_SPAN_NAME_RULES } = require(path.join(lib, 'transform'));
const { SpanMetricsConnector } = require(path.join(lib, 'connector'));

const b64 = (ta) => Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength).toString('base64');

function main(cmd) {
  const real = addonLoader.load();
  const captured = { keyHash: [], startNs: [], endNs: [], traceW0: [], traceW1: [], meta: [] };
  const flushes = [];
  // pass-through wrapper that records what crossed the N-API boundary
  const addon = Object.create(real);
  addon.ingest = (h, b) => {
    for (const k of Object.keys(captured)) captured[k].push(b[k].slice());
    return real.ingest(h, b);
  };
  addon.flush = (h) => {
    const r = real.flush(h);
    flushes.push({ status: r.status, n: r.nSeries, nb: r.nBuckets, key_hash: b64(r.keyHash),
      bucket_counts: b64(r.bucketCounts), sum_ns: b64(r.sumNs), sum: b64(r.sum) });
    return r;
  };
  let t = 1700000000000000000n;
  // native: request bytes through the addon's columnizer (sa_ingest from C++);
  // otherwise decoded in JavaScript and ingested through addon.ingest (captured)
  const native = cmd.native !== false;
  const conn = new SpanMetricsConnector(cmd.config || {}, { addon, clock: () => (t += 1000000000n),
    rules: DEMO_SPAN_NAME_RULES, native });
  const metrics = [];
  const exportsAfter = new Set(cmd.exports_after || []);
  // batch: the requests between exports go through consumeTracesBatch together
  // (the pipeline queue's path: decoded on the columnizer's worker threads)
  let pending = [];
  cmd.requests.forEach((r, i) => {
    const bytes = Buffer.from(r, 'base64');
    if (cmd.batch) pending.push(bytes);
    else conn.consumeTraces(native ? bytes : otlp.decodeTraces(bytes));
    if (cmd.batch && (exportsAfter.has(i) || i === cmd.requests.length - 1)) {
      const errs = conn.consumeTracesBatch(pending);
      if (errs.some(Boolean)) throw errs.find(Boolean);
      pending = [];
    }
    if (exportsAfter.has(i)) metrics.push(otlp.encodeMetrics(conn.exportMetrics()).toString('base64'));
  });
  metrics.push(otlp.encodeMetrics(conn.exportMetrics()).toString('base64'));
  const windows = [];
  const nw = BigInt(conn.cfg.nWindows);
  for (let w = conn.windowBase; w !== null && w < conn.windowBase + nw; w++) {
    const s = conn.windowSketch(w);
    windows.push({ window_id: w.toString(), hll: b64(s.raw.hll), cms: b64(s.raw.cms),
      distinct: Object.fromEntries(s.distinct) });
  }
  const columns = {};
  for (const k of Object.keys(captured)) {
    const parts = captured[k];
    const n = parts.reduce((a, p) => a + p.length, 0);
    const out = k === 'meta' ? new Uint32Array(n) : new BigUint64Array(n);
    let o = 0;
    for (const p of parts) { out.set(p, o); o += p.length; }
    columns[k] = b64(out);
  }
  const st = conn.stats();
  if (native !== (st.nativeRequests > 0) || (native && st.jsRequests)) throw new Error('wrong columnizer path');
  const stats = {};
  for (const [k, v] of Object.entries(st)) stats[k] = typeof v === 'bigint' ? v.toString() : v;
  const services = Object.fromEntries(conn.services);
  conn.shutdown();
  return { columns, flushes, metrics, windows, stats, services,
    window_base: conn.windowBase === null ? null : conn.windowBase.toString() };
}

let input = '';
process.stdin.setEncoding('utf8');
process.stdin.on('data', (c) => { input += c; });
process.stdin.on('end', () => {
  process.stdout.write(JSON.stringify(main(JSON.parse(input))));
});
