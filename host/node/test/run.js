'use strict';
/**
 * CPU tests of the Node host (no GPU needed): OTLP codec round trips, the
 * transform rules, key building, config parsing, the addon's pure helpers and
 * error path, and the connector's host logic (resources, temporality, LRU
 * eviction, A1/A10/A12) over a test-only stand-in for the addon.
 *
 * Run: node test/run.js   (exit code 1 on the first failing test)
 */
const assert = require('assert');
const path = require('path');

const lib = path.join(__dirname, '..', 'lib');
const otlp = require(path.join(lib, 'otlp'));
const keys = require(path.join(lib, 'keys'));
const { applyRules, DEMO_SPAN_NAME_RULES } = require(path.join(lib, 'transform'));
const { SpanMetricsConnector, parseDurationNs, normalizeConfig } = require(path.join(lib, 'connector'));
const { FakeAddon } = require('./fake_addon');

const tests = [];
const test = (name, fn) => tests.push({ name, fn });
const str = (value) => ({ type: 'string', value });

function span(name, opts = {}) {
  return Object.assign({ traceId: Uint8Array.from({ length: 16 }, (_, i) => i + 1),
    spanId: new Uint8Array(8).fill(7), name, kind: 2,
    startTimeUnixNano: 1000000000000n, endTimeUnixNano: 1000003000000n,
    attributes: [], status: { code: 0, message: '' } }, opts);
}
function request(resources) {
  return { resourceSpans: resources.map(([attrs, spans]) => ({
    resource: { attributes: Object.entries(attrs).map(([key, v]) => ({ key,
      value: typeof v === 'object' ? v : str(v) })) },
    scopeSpans: [{ scope: { name: 'test' }, spans }] })) };
}

// ------------------------------------------------------------------ OTLP

test('otlp traces round trip keeps every field the connector reads', () => {
  const req = request([[{ 'service.name': 'frontend', 'k8s.pod.name': 'p-1' }, [
    span('GET /api/cart', { kind: 3, status: { code: 2, message: 'boom' },
      attributes: [{ key: 'http.route', value: str('/api/cart') },
        { key: 'n', value: { type: 'int', value: -42n } },
        { key: 'f', value: { type: 'double', value: 0.25 } },
        { key: 'b', value: { type: 'bool', value: false } },
        { key: 'arr', value: { type: 'array', value: [str('x'), { type: 'int', value: 3n }] } },
        { key: 'kv', value: { type: 'kvlist', value: [{ key: 'a', value: str('b') }] } },
        { key: 'raw', value: { type: 'bytes', value: Uint8Array.from([0, 255]) } }] })]]]);
  const dec = otlp.decodeTraces(otlp.encodeTraces(req));
  const s = dec.resourceSpans[0].scopeSpans[0].spans[0];
  assert.strictEqual(s.name, 'GET /api/cart');
  assert.strictEqual(s.kind, 3);
  assert.deepStrictEqual(s.status, { code: 2, message: 'boom' });
  assert.strictEqual(s.startTimeUnixNano, 1000000000000n);
  assert.strictEqual(s.endTimeUnixNano, 1000003000000n);
  assert.deepStrictEqual(Array.from(s.traceId), Array.from({ length: 16 }, (_, i) => i + 1));
  assert.deepStrictEqual(s.attributes[1].value, { type: 'int', value: -42n });
  assert.deepStrictEqual(s.attributes[4].value.value[1], { type: 'int', value: 3n });
  assert.deepStrictEqual(Array.from(s.attributes[6].value.value), [0, 255]);
  assert.strictEqual(dec.resourceSpans[0].resource.attributes[1].value.value, 'p-1');
});

test('otlp decoder skips unknown fields and rejects truncation', () => {
  const w = new otlp.Writer();
  w.tag(99, 0).varint(5);            // unknown varint
  w.tag(98, 2).string('ignored');    // unknown length-delimited
  const body = otlp.encodeTraces(request([[{ 'service.name': 's' }, [span('a')]]]));
  const buf = Buffer.concat([w.finish(), body]);
  assert.strictEqual(otlp.decodeTraces(buf).resourceSpans.length, 1);
  assert.throws(() => otlp.decodeTraces(body.subarray(0, body.length - 3)), /truncated/);
  assert.deepStrictEqual(otlp.decodeTraces(Buffer.alloc(0)), { resourceSpans: [] });
});

test('otlp metrics encode/decode round trip (sum, histogram, gauge)', () => {
  const req = { resourceMetrics: [{ resource: { attributes: [{ key: 'service.name', value: str('x') }] },
    scopeMetrics: [{ scope: { name: 'spanmetricsconnector' }, metrics: [
      { name: 'calls', sum: { aggregationTemporality: 2, isMonotonic: true,
        dataPoints: [{ attributes: [], startTimeUnixNano: 5n, timeUnixNano: 9n, asInt: 12n }] } },
      { name: 'duration', unit: 'ms', histogram: { aggregationTemporality: 1, dataPoints: [{
        attributes: [{ key: 'span.name', value: str('a') }], startTimeUnixNano: 5n, timeUnixNano: 9n,
        count: 3n, sum: 0, bucketCounts: [0n, 3n], explicitBounds: [2.5] }] } },
      { name: 'g', gauge: { dataPoints: [{ attributes: [], startTimeUnixNano: 1n, timeUnixNano: 2n, asDouble: 1.5 }] } },
    ] }] }] };
  const d = otlp.decodeMetrics(otlp.encodeMetrics(req));
  const [calls, dur, g] = d.resourceMetrics[0].scopeMetrics[0].metrics;
  assert.strictEqual(calls.sum.dataPoints[0].asInt, 12n);
  assert.strictEqual(calls.sum.isMonotonic, true);
  assert.strictEqual(dur.histogram.aggregationTemporality, 1);
  assert.strictEqual(dur.histogram.dataPoints[0].sum, 0);  // optional sum keeps presence
  assert.deepStrictEqual(dur.histogram.dataPoints[0].bucketCounts, [0n, 3n]);
  assert.deepStrictEqual(dur.histogram.dataPoints[0].explicitBounds, [2.5]);
  assert.strictEqual(g.gauge.dataPoints[0].asDouble, 1.5);
});

test('otlp exponential histogram round trip (negative scale/offset, zero count, min/max)', () => {
  const dp = { attributes: [{ key: 'span.name', value: str('a') }], startTimeUnixNano: 5n, timeUnixNano: 9n,
    count: 7n, sum: 12.5, scale: -3, zeroCount: 2n, positive: { offset: -17, bucketCounts: [1n, 0n, 300n] },
    min: 0, max: 9.75 };
  const req = { resourceMetrics: [{ resource: { attributes: [] }, scopeMetrics: [{ scope: { name: 's' },
    metrics: [{ name: 'duration', unit: 'ms', exponentialHistogram: { aggregationTemporality: 2, dataPoints: [dp] } }] }] }] };
  const m = otlp.decodeMetrics(otlp.encodeMetrics(req)).resourceMetrics[0].scopeMetrics[0].metrics[0];
  assert.strictEqual(m.exponentialHistogram.aggregationTemporality, 2);
  const d = m.exponentialHistogram.dataPoints[0];
  assert.deepStrictEqual([d.count, d.sum, d.scale, d.zeroCount, d.min, d.max], [7n, 12.5, -3, 2n, 0, 9.75]);
  assert.deepStrictEqual(d.positive, { offset: -17, bucketCounts: [1n, 0n, 300n] });
  assert.deepStrictEqual(d.negative, { offset: 0, bucketCounts: [] });
});

test('expo restatement (test/expo_ref.js) matches the golden go-expohisto vectors', () => {
  const kat = JSON.parse(require('fs').readFileSync(path.join(__dirname, '..', '..', '..', 'tests', 'golden',
    'expo_kat.json'), 'utf8'));
  const { goLog, mapToIndex, Histogram } = require('./expo_ref');
  for (const [x, y] of kat.go_log) assert.strictEqual(goLog(parseHexFloat(x)), parseHexFloat(y), x);
  for (const [d, sc, i] of kat.map_to_index_ms) assert.strictEqual(mapToIndex(d / 1e6, sc), i, `${d} ${sc}`);
  for (const c of kat.cases) {
    const h = new Histogram(c.max_size), div = c.unit === 's' ? 1e9 : 1e6;
    for (const d of c.durations_ns) h.update(d / div);
    const b = h.buckets(), e = c.expected;
    assert.deepStrictEqual([Number(h.count), Number(h.zero), h.scale, b.offset, b.counts.map(Number)],
      [e.count, e.zero_count, e.scale, e.offset, e.counts], c.name);
    assert.strictEqual(h.sum, parseHexFloat(e.sum), c.name);
  }
});

/** Python float.hex() text -> Number. */
function parseHexFloat(h) {
  const m = /^(-?)0x([01])\.([0-9a-f]*)p([+-]\d+)$/.exec(h);
  if (!m) throw new Error(`bad hex float ${h}`);
  const frac = m[3] ? Number.parseInt(m[3], 16) / 2 ** (4 * m[3].length) : 0;
  const v = (Number(m[2]) + frac) * 2 ** Number(m[4]);
  return m[1] ? -v : v;
}

// ------------------------------------------------------------- transform

test('demo transform rules (A12)', () => {
  assert.strictEqual(applyRules('GET /api/products/0PUK6V6EV0?x=1', DEMO_SPAN_NAME_RULES),
    'GET /api/products/{productId}');
  assert.strictEqual(applyRules('GET /api/cart?sessionId=1', DEMO_SPAN_NAME_RULES), 'GET /api/cart');
  assert.strictEqual(applyRules('POST /api/products/1', DEMO_SPAN_NAME_RULES), 'POST /api/products/1');
  assert.strictEqual(applyRules('GET /api/products/', DEMO_SPAN_NAME_RULES), 'GET /api/products/{productId}');
});

// ------------------------------------------------------------- keys

test('buildKey skips missing dims with no separator (A5) and uses AsString (A6)', () => {
  const dims = [{ name: 'A' }, { name: 'B' }];
  const k1 = keys.buildKeyString('svc', 'op', 2, 0, dims, new Map([['A', str('x')]]));
  const k2 = keys.buildKeyString('svc', 'op', 2, 0, dims, new Map([['B', str('x')]]));
  assert.strictEqual(k1, k2);
  assert.strictEqual(k1, 'svc\0op\0SPAN_KIND_SERVER\0STATUS_CODE_UNSET\0x');
  const ki = keys.buildKeyString('s', 'o', 9, 7, [{ name: 'c' }], new Map([['c', { type: 'int', value: 200n }]]));
  assert.strictEqual(ki, ['s', 'o', '', '', '200'].join('\u0000'));  // A7: out-of-range enums -> ""
});

test('Go FormatFloat(f, -1) for double dimension values', () => {
  assert.strictEqual(keys.formatFloat(1e21), '1000000000000000000000');
  assert.strictEqual(keys.formatFloat(1.5e-7), '0.00000015');
  assert.strictEqual(keys.formatFloat(3), '3');
  assert.strictEqual(keys.formatFloat(-0.1), '-0.1');
});

// ------------------------------------------------------------- config

test('config: durations, defaults and validation', () => {
  assert.strictEqual(parseDurationNs('2ms'), 2e6);
  assert.strictEqual(parseDurationNs('1m30s'), 90e9);
  assert.strictEqual(parseDurationNs('1.5s'), 1.5e9);
  assert.throws(() => parseDurationNs('5 parsecs'));
  const fa = new FakeAddon();
  const c = normalizeConfig({}, fa);
  assert.deepStrictEqual(c.bounds, fa.configDefault().bounds);
  assert.strictEqual(c.namespace, 'traces.span.metrics');
  const c2 = normalizeConfig({ histogram: { unit: 's', explicit: { buckets: ['100ms', '1s', 2] } } }, fa);
  assert.deepStrictEqual(c2.bounds, [0.1, 1, 2]);
  assert.throws(() => normalizeConfig({ histogram: { unit: 'us' } }, fa));
  assert.throws(() => normalizeConfig({ aggregation_temporality: 'X' }, fa));
  assert.strictEqual(normalizeConfig({ histogram: { exponential: {} } }, fa).expMaxSize, 160);
  assert.strictEqual(normalizeConfig({ histogram: { exponential: { max_size: 40 } } }, fa).expMaxSize, 40);
  assert.strictEqual(c.expMaxSize, 0);
  assert.throws(() => normalizeConfig({ histogram: { exponential: {}, explicit: { buckets: [1] } } }, fa), /either/);
  assert.throws(() => normalizeConfig({ histogram: { exponential: { max_size: 1 } } }, fa), /max_size/);
});

// ------------------------------------------------------------- addon

test('addon loads; pure helpers work; engine errors carry sa_status codes', () => {
  const addon = require('../lib/addon').load();
  assert.strictEqual(addon.abiVersion(), 4);
  const d = addon.configDefault();
  assert.deepStrictEqual(d.bounds, [2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000]);
  const t = addon.bucketThresholds(d.bounds, 'ms');
  assert.strictEqual(t.nNeg, 0);
  assert.deepStrictEqual(Array.from(t.thresholds), d.bounds.map((b) => BigInt(b) * 1000000n));
  assert.throws(() => addon.bucketThresholds([3, 2], 'ms'), (e) => e.code === addon.status.EINVAL);
  assert.strictEqual(addon.hllEstimate(new Uint8Array(1 << 14), 14), 0);
  assert.throws(() => addon.hllEstimate(new Uint8Array(10), 14), (e) => e.code === addon.status.EINVAL);
  assert.throws(() => addon.create({ cmsW: 1000 }), (e) => e.code === addon.status.EINVAL ||
    e.code === addon.status.EDEVICE);
  assert.throws(() => addon.ingest({}, {}), TypeError);
  let h = null;
  try {
    h = addon.create({});
  } catch (e) {
    assert.strictEqual(e.code, addon.status.EDEVICE);  // no GPU here: fails loudly, no fallback
  }
  if (h) {  // a GPU is visible: the handle works until destroyed
    assert.strictEqual(addon.stats(h).spans, 0n);
    addon.destroy(h);
    assert.throws(() => addon.stats(h), (e) => e.code === addon.status.ESTATE);
  }
});

// ------------------------------------------------------------- connector (host logic)

function mkConnector(cfg = {}, t = { now: 1000n }) {
  const addon = new FakeAddon();
  const conn = new SpanMetricsConnector(Object.assign({ batch_size: 4 }, cfg), { addon, clock: () => t.now });
  return { conn, addon, t };
}
const dpsOf = (req, metric) => req.resourceMetrics.flatMap((rm) => rm.scopeMetrics[0].metrics
  .filter((m) => m.name === metric).flatMap((m) => (m.sum || m.histogram || m.gauge).dataPoints
    .map((dp) => Object.assign({ resource: rm.resource }, dp))));
const attr = (dp, k) => (dp.attributes.find((a) => a.key === k) || {}).value;

test('connector: A1 skip, A10 resource grouping, calls == histogram count', () => {
  const { conn } = mkConnector();
  conn.consumeTraces(request([
    [{ 'service.name': 'a' }, [span('x'), span('x'), span('y', { status: { code: 2 } })]],
    [{ 'host.name': 'nosvc' }, [span('x')]],                                  // A1
    [{ 'service.name': 'a', 'k8s.pod.name': 'p2' }, [span('x')]],             // A10
  ]));
  const out = conn.exportMetrics();
  assert.strictEqual(out.resourceMetrics.length, 2);
  const calls = dpsOf(out, 'traces.span.metrics.calls');
  const hist = dpsOf(out, 'traces.span.metrics.duration');
  assert.deepStrictEqual(calls.map((d) => d.asInt), [2n, 1n, 1n]);
  assert.deepStrictEqual(hist.map((d) => d.count), [2n, 1n, 1n]);
  assert.strictEqual(attr(calls[1], 'status.code').value, 'STATUS_CODE_ERROR');
  assert.strictEqual(hist[0].sum, 6);   // 2 x 3 ms
  assert.deepStrictEqual(hist[0].bucketCounts.slice(0, 3), [0n, 2n, 0n]);  // 3 ms -> (2,4]
  assert.strictEqual(out.resourceMetrics[0].scopeMetrics[0].scope.name, 'spanmetricsconnector');
  const m = out.resourceMetrics[0].scopeMetrics[0].metrics;
  assert.strictEqual(m[1].unit, 'ms');
  assert.strictEqual(m[0].sum.aggregationTemporality, otlp.AGGREGATION_TEMPORALITY.CUMULATIVE);
});

test('connector: cumulative keeps totals and the resource start time', () => {
  const { conn, t } = mkConnector();
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x')]]]));
  t.now = 2000n;
  conn.exportMetrics();
  t.now = 3000n;
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('z')]]]));
  t.now = 4000n;
  const out = conn.exportMetrics();
  const calls = dpsOf(out, 'traces.span.metrics.calls');
  assert.deepStrictEqual(calls.map((d) => [d.asInt, d.startTimeUnixNano, d.timeUnixNano]),
    [[2n, 1000n, 4000n], [1n, 1000n, 4000n]]);
  t.now = 5000n;
  assert.strictEqual(dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls').length, 2);  // no new data
});

test('connector: delta emits only touched series, start = previous export', () => {
  const { conn, t } = mkConnector({ aggregation_temporality: 'AGGREGATION_TEMPORALITY_DELTA' });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('y')]]]));
  t.now = 2000n;
  let out = conn.exportMetrics();
  assert.deepStrictEqual(dpsOf(out, 'traces.span.metrics.calls').map((d) => [d.asInt, d.startTimeUnixNano]),
    [[1n, 1000n], [1n, 1000n]]);
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('x')]]]));
  t.now = 3000n;
  out = conn.exportMetrics();
  const c = dpsOf(out, 'traces.span.metrics.calls');
  assert.deepStrictEqual(c.map((d) => [attr(d, 'span.name').value, d.asInt, d.startTimeUnixNano, d.timeUnixNano]),
    [['x', 2n, 2000n, 3000n]]);
  assert.strictEqual(dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls').length, 0);
});

test('connector: engine drops (SA_EFULL) are counted and reported, never silent', () => {
  const seen = [];
  const addon = new FakeAddon();
  const conn = new SpanMetricsConnector({ batch_size: 4 }, { addon, clock: () => 1000n, onDrop: (i) => seen.push(i) });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x')]]]));
  const flush = addon.flush.bind(addon);
  addon.flush = () => Object.assign(flush(), { status: addon.status.EFULL });
  addon.dropped = 7n;
  conn.exportMetrics();
  assert.deepStrictEqual(seen.map((i) => [i.droppedSpans, i.droppedFlushes]), [[7n, 1]]);
  assert.strictEqual(conn.stats().droppedSpans, 7n);
});

test('connector: resource LRU evicts, exports the evicted once, then forgets it', () => {
  const { conn, t } = mkConnector({ resource_metrics_cache_size: 1 });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x')]],
    [{ 'service.name': 'b' }, [span('x')]]]));
  let out = conn.exportMetrics();
  assert.strictEqual(out.resourceMetrics.length, 2);   // b live, a evicted but still exported
  out = conn.exportMetrics();
  assert.strictEqual(out.resourceMetrics.length, 1);   // a dropped after that export
  t.now = 9000n;
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x')]]]));
  out = conn.exportMetrics();
  const a = dpsOf(out, 'traces.span.metrics.calls').filter((d) => attr(d, 'service.name').value === 'a');
  assert.deepStrictEqual(a.map((d) => [d.asInt, d.startTimeUnixNano]), [[1n, 9000n]]);  // fresh start
});

test('connector: dimensions, defaults, exclude_dimensions and first-seen attribute types', () => {
  const { conn } = mkConnector({ dimensions: [{ name: 'http.status_code' }, { name: 'region', default: 'eu' }],
    exclude_dimensions: ['span.kind'] });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [
    span('x', { attributes: [{ key: 'http.status_code', value: { type: 'int', value: 200n } }] }),
    span('x', { attributes: [{ key: 'http.status_code', value: str('200') }] }),   // A6: same key
    span('x')]]]));
  const c = dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls');
  assert.strictEqual(c.length, 2);
  assert.strictEqual(c[0].asInt, 2n);
  assert.deepStrictEqual(attr(c[0], 'http.status_code'), { type: 'int', value: 200n });  // first seen
  assert.deepStrictEqual(attr(c[0], 'region'), str('eu'));
  assert.strictEqual(attr(c[0], 'span.kind'), undefined);
  assert.strictEqual(attr(c[1], 'http.status_code'), undefined);
});

// connector options restated in tests/golden/gen_golden.py (connector_cases)
const KAT = require(path.join(__dirname, '..', '..', '..', 'tests', 'golden', 'spanmetrics_kat.json'));
const katCase = (name) => KAT.connector_cases.find((c) => c.name === name);
const dpKey = (dp) => JSON.stringify(dp.attributes.map((a) => [a.key, a.value.value]));

test('connector: metrics_expiration drops resources not seen within it, after one last export (KAT)', () => {
  const c = katCase('metrics_expiration');
  const t = { now: 0n };
  const { conn } = mkConnector(c.config, t);
  const got = [];
  for (const op of c.ops) {
    t.now = BigInt(op.t);
    if (op.consume) {
      conn.consumeTraces(request(op.consume.map(([svc, n]) => [{ 'service.name': svc },
        Array.from({ length: n }, () => span('op'))])));
    } else {
      const e = {};
      for (const dp of dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls')) {
        e[attr(dp, 'service.name').value] = [Number(dp.asInt), Number(dp.startTimeUnixNano)];
      }
      got.push(e);
    }
  }
  assert.deepStrictEqual(got, c.expected);
});

for (const name of ['calls_and_histogram_dimensions', 'histogram_disable']) {
  test(`connector: ${name.replace(/_/g, ' ')} (KAT)`, () => {
    const c = katCase(name);
    const { conn } = mkConnector(c.config);
    for (const [svc, nm, kind, st, attrs] of c.spans) {
      conn.consumeTraces(request([[{ 'service.name': svc }, [span(nm, { kind, status: { code: st, message: '' },
        attributes: Object.entries(attrs).map(([key, v]) => ({ key, value: str(v) })) })]]]));
    }
    const out = conn.exportMetrics();
    const calls = dpsOf(out, 'traces.span.metrics.calls').map((dp) => [dpKey(dp), Number(dp.asInt)]).sort();
    const hist = dpsOf(out, 'traces.span.metrics.duration').map((dp) => [dpKey(dp), Number(dp.count)]).sort();
    const want = (l) => l.map(([at, n]) => [JSON.stringify(at), n]).sort();
    assert.deepStrictEqual(calls, want(c.expected.calls));
    assert.deepStrictEqual(hist, want(c.expected.histogram));
    if (name === 'histogram_disable') {
      assert.ok(out.resourceMetrics.every((rm) => rm.scopeMetrics[0].metrics.every((m) => !m.histogram)));
    } else {
      // the sketches see each span once: every count-min row holds the
      // window's ERROR spans once, and the heavy hitters are the histogram
      // series (never the calls series too); the engine's span count is the
      // spans', its second (calls) records taken out
      const w = conn.windowSketch(Number(span('x').endTimeUnixNano / 10000000000n));
      for (let j = 0; j < w.raw.cmsD; j++) {
        const row = w.raw.cms.subarray(j * w.raw.cmsW, (j + 1) * w.raw.cmsW);
        assert.strictEqual(row.reduce((a, x) => a + x, 0), c.expected.window_error_spans);
      }
      const top = w.topErrors().map((e) => [JSON.stringify(e.attributes.map((a) => [a.key, a.value.value])), e.errors]);
      assert.deepStrictEqual(top.sort(), want(c.expected.top_errors));
      const st = conn.stats();
      assert.strictEqual(st.spans, BigInt(c.spans.length));
      assert.strictEqual(st.callsRecords, c.spans.length);
      assert.strictEqual(st.invalidService, 0n);
    }
  });
}

test('connector: include_instrumentation_scope keys listed scopes by name and version (KAT)', () => {
  const c = katCase('include_instrumentation_scope');
  const want = c.expected.calls.map(([at, n]) => [JSON.stringify(at), n]).sort();
  // decoded requests, and the same spans as OTLP bytes (the scope goes
  // through the decoder; the option keeps the JavaScript columnizer)
  for (const bytes of [false, true]) {
    const { conn } = mkConnector(c.config);
    for (const [svc, nm, kind, st, attrs, sn, sv] of c.spans) {
      const req = { resourceSpans: [{ resource: { attributes: [{ key: 'service.name', value: str(svc) }] },
        scopeSpans: [{ scope: { name: sn, version: sv }, spans: [span(nm, { kind, status: { code: st, message: '' },
          attributes: Object.entries(attrs).map(([key, v]) => ({ key, value: str(v) })) })] }] }] };
      conn.consumeTraces(bytes ? otlp.encodeTraces(req) : req);
    }
    const out = conn.exportMetrics();
    const calls = dpsOf(out, 'traces.span.metrics.calls').map((dp) => [dpKey(dp), Number(dp.asInt)]).sort();
    assert.deepStrictEqual(calls, want);
    const hist = dpsOf(out, 'traces.span.metrics.duration').map((dp) => [dpKey(dp), Number(dp.count)]).sort();
    assert.deepStrictEqual(hist, want);
  }
});

test('connector: consumes OTLP bytes; columns carry trace ids and meta bits', () => {
  const { conn, addon } = mkConnector({ batch_size: 2 });
  const tid = Uint8Array.from({ length: 16 }, (_, i) => 0xA0 + i);
  conn.consumeTraces(otlp.encodeTraces(request([[{ 'service.name': 'a' }, [
    span('x', { traceId: tid, kind: 4, status: { code: 2 } }), span('y', { kind: 11 })]]])));
  assert.strictEqual(addon.batches.length, 1);   // batch_size reached -> one ingest
  const b = addon.batches[0];
  assert.strictEqual(b.traceW0[0], Buffer.from(tid).readBigUInt64LE(0));
  assert.strictEqual(b.traceW1[0], Buffer.from(tid).readBigUInt64LE(8));
  assert.strictEqual(b.meta[0], 0 | (4 << 16) | (2 << 19));
  assert.strictEqual(b.meta[1], 0 | (7 << 16));   // out-of-range kind clamps into the 3-bit field
});

test('connector: window ring follows the data and sketch metrics are emitted once', () => {
  const { conn, addon } = mkConnector({ sketches: { emit: true, n_windows: 4 } });
  const W = 10000000000n;
  const at = (w, name, code = 0) => span(name, { startTimeUnixNano: w * W + 1n, endTimeUnixNano: w * W + 5n,
    status: { code } });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [at(100n, 'x'), at(101n, 'x', 2)]]]));
  let out = conn.exportMetrics();
  assert.strictEqual(addon.base, 98n);                   // base = max window - (n_windows - 1)
  // window 101 is still open (the newest one seen); window 100 is closed
  assert.deepStrictEqual(dpsOf(out, 'traces.span.metrics.window.distinct_traces')
    .map((x) => [x.startTimeUnixNano / W, x.asDouble > 0]), [[100n, true]]);
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [at(110n, 'x')]]]));
  out = conn.exportMetrics();
  assert.strictEqual(addon.base, 107n);                  // 101 was read before it was retired
  const d = dpsOf(out, 'traces.span.metrics.window.distinct_traces');
  assert.deepStrictEqual(d.map((x) => x.startTimeUnixNano / W), [101n]);
  const e = dpsOf(out, 'traces.span.metrics.window.errors');
  assert.deepStrictEqual(e.map((x) => [x.startTimeUnixNano / W, x.asInt]), [[101n, 1n]]);
  assert.strictEqual(dpsOf(conn.exportMetrics(), 'traces.span.metrics.window.distinct_traces').length, 0);
});

test('connector: aggregation_cardinality_limit folds new keys into one overflow series', () => {
  const { conn } = mkConnector({ aggregation_cardinality_limit: 2 });
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('y'), span('z'), span('w'),
    span('x')]], [{ 'service.name': 'b' }, [span('q')]]]));
  const c = dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls');
  const a = c.filter((d) => d.resource.attributes[0].value.value === 'a');
  assert.deepStrictEqual(a.map((d) => d.asInt), [2n, 1n, 2n]);
  assert.deepStrictEqual(a[2].attributes, [{ key: 'otel.metric.overflow', value: { type: 'bool', value: true } }]);
  assert.strictEqual(c.length, 4);   // the limit is per resource
});

test('connector: events metric counts span events per key + event dimensions', () => {
  const { conn, addon } = mkConnector({ events: { enabled: true, dimensions: [{ name: 'exception.type' }] } });
  const ev = (t) => ({ timeUnixNano: 5n, name: 'exception', attributes: t ? [{ key: 'exception.type', value: str(t) }] : [] });
  conn.consumeTraces(otlp.encodeTraces(request([[{ 'service.name': 'a' }, [
    span('x', { events: [ev('IOError'), ev('IOError'), ev('Timeout')] }), span('x', { events: [ev(null)] })]]])));
  const out = conn.exportMetrics();
  const e = dpsOf(out, 'traces.span.metrics.events');
  assert.deepStrictEqual(e.map((d) => [(attr(d, 'exception.type') || {}).value, d.asInt]),
    [['IOError', 2n], ['Timeout', 1n], [undefined, 1n]]);
  assert.strictEqual(attr(e[0], 'span.name').value, 'x');
  assert.deepStrictEqual(dpsOf(out, 'traces.span.metrics.calls').map((d) => d.asInt), [2n]);
  assert.strictEqual(conn.stats().eventRecords, 4);
  const metas = addon.batches.flatMap((b) => Array.from(b.meta));
  assert.strictEqual(metas.filter((m) => m === 0xFFFF).length, 4);  // no sketch for event records
});

test('connector: exemplars carry trace/span ids and the duration, one export interval each', () => {
  const { conn } = mkConnector({ exemplars: { enabled: true, max_per_data_point: 2 } });
  const tid = Uint8Array.from({ length: 16 }, (_, i) => 0x10 + i);
  conn.consumeTraces(request([[{ 'service.name': 'a' }, [span('x', { traceId: tid }), span('x'), span('x')]]]));
  let out = conn.exportMetrics();
  let h = dpsOf(out, 'traces.span.metrics.duration')[0];
  assert.strictEqual(h.exemplars.length, 2);
  assert.deepStrictEqual(Array.from(h.exemplars[0].traceId), Array.from(tid));
  assert.strictEqual(h.exemplars[0].asDouble, 3);
  const dec = otlp.decodeMetrics(otlp.encodeMetrics(out));
  const hd = dec.resourceMetrics[0].scopeMetrics[0].metrics[1].histogram.dataPoints[0];
  assert.strictEqual(hd.exemplars.length, 2);
  assert.deepStrictEqual(Array.from(hd.exemplars[0].traceId), Array.from(tid));
  assert.strictEqual(hd.exemplars[0].timeUnixNano, 1000003000000n);
  out = conn.exportMetrics();
  h = dpsOf(out, 'traces.span.metrics.duration')[0];
  assert.strictEqual(h.exemplars, undefined);
});

// ------------------------------------------------- native columnizer vs JavaScript

function expoDps(req) {
  return req.resourceMetrics.flatMap((rm) => rm.scopeMetrics[0].metrics
    .filter((m) => m.exponentialHistogram).flatMap((m) => m.exponentialHistogram.dataPoints));
}

for (const temporality of ['AGGREGATION_TEMPORALITY_CUMULATIVE', 'AGGREGATION_TEMPORALITY_DELTA']) {
  test(`connector: exponential histograms, ${temporality.slice(24).toLowerCase()} (host fold == one go-expohisto)`, () => {
    const { Histogram } = require('./expo_ref');
    const maxSize = 6;
    const { conn, t } = mkConnector({ aggregation_temporality: temporality, histogram: { exponential: { max_size: maxSize } } });
    const cumulative = temporality.endsWith('CUMULATIVE');
    let rng = 12345;
    const rand = () => { rng = (rng * 1103515245 + 12345) % 2147483648; return rng / 2147483648; };
    const all = new Map([['x', new Histogram(maxSize)], ['y', new Histogram(maxSize)]]);
    let mixedScales = 0;  // folds of a delta whose scale differs from the running histogram's
    for (let round = 0; round < 4; round++) {
      const interval = new Map([['x', new Histogram(maxSize)], ['y', new Histogram(maxSize)]]);
      const spans = [];
      for (let i = 0; i < 40; i++) {
        const name = i % 3 ? 'x' : 'y';
        // each round widens the range on a different side, forcing host-side downscales
        const ns = i === 7 ? 0 : Math.round(Math.exp(rand() * (2 + round) + (round % 2 ? 10 : 16 - round)));
        spans.push(span(name, { startTimeUnixNano: 1000000000000n, endTimeUnixNano: 1000000000000n + BigInt(ns) }));
        all.get(name).update(ns / 1e6);
        interval.get(name).update(ns / 1e6);
      }
      for (const [k, h] of interval) mixedScales += round > 0 && h.scale !== all.get(k).scale;
      conn.consumeTraces(request([[{ 'service.name': 'a' }, spans]]));
      t.now += 1000n;
      const out = otlp.decodeMetrics(otlp.encodeMetrics(conn.exportMetrics()));
      const dps = expoDps(out);
      assert.strictEqual(dps.length, 2);
      for (const dp of dps) {
        const name = attr(dp, 'span.name').value;
        const h = (cumulative ? all : interval).get(name), b = h.buckets();
        assert.deepStrictEqual([dp.count, dp.zeroCount, dp.scale, dp.positive.offset, dp.positive.bucketCounts],
          [h.count, h.zero, h.scale, b.offset, b.counts], `${name} round ${round}`);
        assert.strictEqual(dp.min, h.min);
        assert.strictEqual(dp.max, h.max);
        assert.ok(Math.abs(dp.sum - h.sum) <= 1e-9 * h.sum);
      }
      const calls = dpsOf(out, 'traces.span.metrics.calls');
      assert.deepStrictEqual(calls.map((d) => d.asInt).sort(), dps.map((d) => d.count).sort());
    }
    assert.ok(mixedScales >= 3, `fold exercised ${mixedScales} scale changes`);
  });
}

const { NativeColumnizerFakeAddon } = require('./fake_addon');

function mixedRequests() {
  const tid = (k) => Uint8Array.from({ length: 16 }, (_, i) => (i * 7 + k) & 255);
  const W = 10000000000n;
  const base = 170000000n * W;
  let k = 0;
  const sp = (name, o = {}) => span(name, Object.assign({ traceId: tid(++k),
    startTimeUnixNano: base + BigInt(k) * 1000003n, endTimeUnixNano: base + BigInt(k) * 1000003n + BigInt(k * 7919 % 50) * 1000000n }, o));
  const reqs = [];
  for (let r = 0; r < 6; r++) {
    reqs.push(request([
      [{ 'service.name': 'frontend', 'k8s.pod.name': `fe-${r % 2}`, 'pid': { type: 'int', value: BigInt(100 + (r % 3)) },
        'ratio': { type: 'double', value: 0.25 }, 'args': { type: 'array', value: [str('node'), { type: 'int', value: 2n }] } }, [
        sp('GET /api/products/0PUK6V6EV0?currencyCode=USD'), sp('GET /api/products/'),
        sp('GET /api/cart?x=1\nsecond?y'), sp('ΣΠΑΝ 😀', { kind: 9, status: { code: 7 } }),
        sp('checkout', { status: { code: 2 }, kind: -1, traceId: new Uint8Array(3),
          attributes: [{ key: 'http.status_code', value: { type: 'int', value: 500n } }] }),
        sp('checkout', { attributes: [{ key: 'http.status_code', value: str('500') },
          { key: 'region', value: { type: 'kvlist', value: [{ key: 'a', value: { type: 'double', value: 1e21 } }] } }] }),
        sp('bytes', { attributes: [{ key: 'http.status_code', value: { type: 'bytes', value: Uint8Array.from([0, 255, 7]) } }] }),
        sp('dbl', { attributes: [{ key: 'http.status_code', value: { type: 'double', value: 1.5e-7 } }] }),
      ]],
      [{ 'host.name': 'no-service' }, [sp('skipped')]],
      [{ 'service.name': { type: 'int', value: 5n } }, [sp('non-string service')]],
      [{ 'service.name': 'cart', 'service.name ': 'x' }, [sp('op-' + r), sp('op-' + r, { kind: 3 })]],
    ]));
  }
  return reqs;
}

function runBoth(cfg, rules, reqs, collide = false, batched = false) {
  const out = [];
  for (const native of [true, false]) {
    const addon = native ? new NativeColumnizerFakeAddon() : new FakeAddon();
    addon.collide = collide;
    addon.batched = batched;
    const t = { now: 1000n };
    const conn = new SpanMetricsConnector(Object.assign({ batch_size: 16 }, cfg),
      { addon, rules, native, clock: () => (t.now += 1n) });
    const exports = [];
    reqs.forEach((r, i) => {
      conn.consumeTraces(otlp.encodeTraces(r));
      if (i % 2 === 1) exports.push(otlp.encodeMetrics(conn.exportMetrics()).toString('hex'));
    });
    exports.push(otlp.encodeMetrics(conn.exportMetrics()).toString('hex'));
    const cols = {};
    for (const c of ['keyHash', 'startNs', 'endNs', 'traceW0', 'traceW1', 'meta']) {
      cols[c] = addon.batches.flatMap((b) => Array.from(b[c]));
    }
    out.push({ exports, cols, stats: conn.stats(), services: [...conn.services] });
  }
  return out;
}

test('native columnizer: same columns and same OTLP metrics as the JavaScript path', () => {
  const reqs = mixedRequests();
  for (const [cfg, rules] of [
    [{}, DEMO_SPAN_NAME_RULES],
    [{ dimensions: [{ name: 'http.status_code' }, { name: 'region', default: 'eu' }, { name: 'k8s.pod.name' },
      { name: 'args' }, { name: 'ratio' }] }, DEMO_SPAN_NAME_RULES],
    [{ exclude_dimensions: ['span.kind', 'status.code'], resource_metrics_key_attributes: ['service.name'] }, []],
    [{ resource_metrics_cache_size: 1, aggregation_temporality: 'AGGREGATION_TEMPORALITY_DELTA' }, DEMO_SPAN_NAME_RULES],
  ]) {
    for (const batched of [false, true]) {  // the columnizer's batched span path (high cardinality) too
      const [nat, js] = runBoth(cfg, rules, reqs, false, batched);
      assert.ok(nat.stats.nativeRequests > 0 && nat.stats.jsRequests === 0, JSON.stringify(cfg));
      assert.strictEqual(js.stats.nativeRequests, 0);
      assert.deepStrictEqual(nat.cols, js.cols, JSON.stringify(cfg));
      assert.deepStrictEqual(nat.exports, js.exports, JSON.stringify(cfg));
      assert.deepStrictEqual(nat.services, js.services);
      assert.strictEqual(nat.stats.nativeRemaps, 0, JSON.stringify(cfg));
    }
  }
});

function eventRequests() {
  const ev = (t, x) => ({ timeUnixNano: 5n, name: 'exception', attributes: [
    ...(t ? [{ key: 'exception.type', value: str(t) }] : []), ...(x ? [{ key: 'x', value: { type: 'int', value: x } }] : [])] });
  const tid = (k) => Uint8Array.from({ length: 16 }, (_, i) => (i * 13 + k) & 255);
  const reqs = [];
  for (let r = 0; r < 6; r++) {
    const spans = [];
    for (let i = 0; i < 9; i++) {
      spans.push(span(`op-${(r * 3 + i) % 7}`, { traceId: tid(r * 9 + i), status: { code: i % 4 === 0 ? 2 : 0 },
        events: i % 3 === 0 ? [] : [ev(i % 2 ? 'IOError' : 'Timeout', BigInt(i % 3)), ...(i === 4 ? [ev(null), ev('IOError')] : [])] }));
    }
    reqs.push(request([[{ 'service.name': `svc-${r % 2}`, 'k8s.pod.name': `p-${r % 3}` }, spans],
      [{ 'service.name': 'other' }, [span('lone', { events: [ev('E', 1n)] })]]]));
  }
  return reqs;
}

test('native columnizer: cardinality limit, exemplars and events == the JavaScript path', () => {
  const reqs = mixedRequests().concat(eventRequests());
  for (const [cfg, rules] of [
    [{ aggregation_cardinality_limit: 3 }, DEMO_SPAN_NAME_RULES],
    [{ aggregation_cardinality_limit: 2, dimensions: [{ name: 'http.status_code' }], resource_metrics_cache_size: 2 }, []],
    [{ exemplars: { enabled: true, max_per_data_point: 2 } }, DEMO_SPAN_NAME_RULES],
    [{ exemplars: { enabled: true, max_per_data_point: 1 }, aggregation_temporality: 'AGGREGATION_TEMPORALITY_DELTA' }, []],
    [{ events: { enabled: true, dimensions: [{ name: 'exception.type' }, { name: 'x', default: 'none' }] } }, DEMO_SPAN_NAME_RULES],
    [{ aggregation_cardinality_limit: 4, dimensions: [{ name: 'k8s.pod.name' }] }, DEMO_SPAN_NAME_RULES],
    [{ events: { enabled: true, dimensions: [{ name: 'exception.type' }] },
      aggregation_cardinality_limit: 4 }, DEMO_SPAN_NAME_RULES],
    // a resource-level dimension with resource identity on service.name only:
    // the signature cache must key on the pod, not on the resource hash
    [{ dimensions: [{ name: 'k8s.pod.name' }, { name: 'http.status_code' }],
      resource_metrics_key_attributes: ['service.name'] }, DEMO_SPAN_NAME_RULES],
    [{ events: { enabled: true, dimensions: [{ name: 'exception.type' }] }, exemplars: { enabled: true, max_per_data_point: 3 },
      aggregation_cardinality_limit: 4, dimensions: [{ name: 'k8s.pod.name' }] }, DEMO_SPAN_NAME_RULES],
  ]) {
    for (const batched of [false, true]) {
    const [nat, js] = runBoth(cfg, rules, reqs, false, batched);
    assert.ok(nat.stats.nativeRequests === reqs.length && nat.stats.jsRequests === 0, `${nat.stats.nativeRequests} ${nat.stats.jsRequests}`);
    assert.deepStrictEqual(nat.cols, js.cols, JSON.stringify(cfg));
    assert.deepStrictEqual(nat.exports, js.exports, JSON.stringify(cfg));
    assert.strictEqual(nat.stats.eventRecords, js.stats.eventRecords);
    assert.strictEqual(nat.stats.nativeRemaps, 0, JSON.stringify(cfg));  // the native side keyed every series as the host does
    if (cfg.events) assert.ok(js.stats.eventRecords > 40);
    }
  }
  // a limited resource really overflows, and exemplars really appear, on the native path
  const [nat] = runBoth({ aggregation_cardinality_limit: 2, exemplars: { enabled: true } }, [], eventRequests());
  const dec = nat.exports.map((h) => otlp.decodeMetrics(Buffer.from(h, 'hex')));
  const calls = dec.flatMap((d) => dpsOf(d, 'traces.span.metrics.calls'));
  assert.ok(calls.some((d) => attr(d, 'otel.metric.overflow')));
  assert.ok(dec.flatMap((d) => dpsOf(d, 'traces.span.metrics.duration')).some((d) => d.exemplars && d.exemplars.length));
});

test('series ids: a 64-bit collision is re-salted on both paths (never thrown), outputs unchanged', () => {
  const reqs = mixedRequests();
  const [natRef, jsRef] = runBoth({}, DEMO_SPAN_NAME_RULES, reqs);
  // every seed-0 id is 42: each new series after the first collides and is re-salted
  const real = keys.seriesHashSeeded;
  keys.seriesHashSeeded = (rh, k, seed) => (seed === 0n ? 42n : real(rh, k, seed));
  let nat, js;
  try {
    [nat, js] = runBoth({}, DEMO_SPAN_NAME_RULES, reqs, true, true);
  } finally {
    keys.seriesHashSeeded = real;
  }
  assert.ok(nat.stats.nativeRequests > 0 && js.stats.collisions > 0);
  assert.deepStrictEqual(nat.cols, js.cols);
  assert.deepStrictEqual(nat.exports, js.exports);
  // the same series, the same spans per series: only the ids moved
  const perId = (cols) => {
    const m = new Map();
    cols.keyHash.forEach((k, i) => m.set(k, (m.get(k) || 0) + 1));
    return [...m.values()].sort((a, b) => a - b);
  };
  assert.deepStrictEqual(perId(js.cols), perId(jsRef.cols));
  assert.strictEqual(new Set(js.cols.keyHash).size, new Set(natRef.cols.keyHash).size);
  // the dictionary: two keys on one seed-0 id get distinct ids
  keys.seriesHashSeeded = (rh, k, seed) => (seed === 0n ? 42n : real(rh, k, seed));
  try {
    const d = new keys.KeyDictionary();
    const a = d.intern(1n, Buffer.from('a'), {}, {}), b = d.intern(1n, Buffer.from('b'), {}, {});
    assert.ok(a === 42n && b !== 42n && b !== 0n && d.collisions === 1);
    assert.strictEqual(d.intern(1n, Buffer.from('b'), {}, {}), b);
  } finally {
    keys.seriesHashSeeded = real;
  }
});

test('native columnizer: consumeTracesBatch on worker threads == consumeTraces one request at a time', () => {
  const reqs = mixedRequests().map((r) => otlp.encodeTraces(r));
  for (let r = 0; r < 12; r++) {  // new series, services and resources appear mid-batch
    reqs.push(otlp.encodeTraces(request([[{ 'service.name': `svc-${r % 5}`, 'k8s.pod.name': `p-${r % 3}` },
      [span(`op-${r % 4}`), span(`op-${r}`, { status: { code: 2 } }), span('GET /api/products/X?y=1')]]])));
  }
  const fallback = Buffer.from(otlp.encodeTraces(request([[{ 'service.name': 'u' }, [span('GET /x\u00e9')]]])));
  fallback[fallback.indexOf(0xC3)] = 0xFF;
  reqs.splice(7, 0, fallback);
  reqs.splice(11, 0, reqs[3].subarray(0, reqs[3].length - 5));  // truncated: rejected
  const rowsOf = (addon) => {
    const rows = [];
    for (const b of addon.batches) {
      for (let i = 0; i < b.keyHash.length; i++) rows.push([b.keyHash[i], b.startNs[i], b.endNs[i], b.traceW0[i], b.traceW1[i], b.meta[i]].join(','));
    }
    return rows.sort();
  };
  for (const r of eventRequests().concat(eventRequests())) reqs.push(otlp.encodeTraces(r));  // the second time: nothing new
  for (const cfg of [{}, { dimensions: [{ name: 'http.status_code' }, { name: 'k8s.pod.name' }] },
    { resource_metrics_cache_size: 2 },
    { aggregation_cardinality_limit: 3, exemplars: { enabled: true }, events: { enabled: true, dimensions: [{ name: 'exception.type' }] } },
    { events: { enabled: true, dimensions: [{ name: 'exception.type' }] } }]) {
    const out = [];
    for (const threads of [1, 4, -4]) {  // -4: four threads, the batched span path forced
      const addon = new NativeColumnizerFakeAddon();
      addon.batched = threads < 0;
      const t = { now: 1000n };
      const conn = new SpanMetricsConnector(Object.assign({ batch_size: 16, columnizer_threads: Math.abs(threads) }, cfg),
        { addon, rules: DEMO_SPAN_NAME_RULES, clock: () => (t.now += 1n) });
      let errs;
      if (threads === 1) {
        errs = reqs.map((r) => { try { conn.consumeTraces(r); return null; } catch (e) { return e; } });
      } else {
        errs = conn.consumeTracesBatch(reqs.slice(0, 9)).concat(conn.consumeTracesBatch(reqs.slice(9)));
      }
      const exp = otlp.encodeMetrics(conn.exportMetrics()).toString('hex');
      out.push({ errs: errs.map((e) => (e ? 'error' : null)), rows: rowsOf(addon), exp, services: [...conn.services],
        stats: conn.stats() });
    }
    const [one, batch, batched] = out;
    assert.deepStrictEqual(batched, batch, JSON.stringify(cfg));
    assert.strictEqual(one.errs.filter(Boolean).length, 1);
    assert.deepStrictEqual(batch.errs, one.errs, JSON.stringify(cfg));
    assert.deepStrictEqual(batch.rows, one.rows, JSON.stringify(cfg));
    assert.deepStrictEqual(batch.exp, one.exp, JSON.stringify(cfg));
    assert.deepStrictEqual(batch.services, one.services);
    assert.strictEqual(batch.stats.jsRequests, 1);  // the non-UTF-8 request
    assert.strictEqual(batch.stats.eventRecords, one.stats.eventRecords);
    assert.strictEqual(batch.stats.nativeRequests, one.stats.nativeRequests);
  }
});

test('native columnizer: after a threaded batch, a forget or remap is seen by single-request calls', () => {
  // the threaded batch fills the columnizer's shared signature cache; an LRU
  // eviction (columnizerForget at export) or a collision remap then changes
  // the series its entries name, and a later one-request call must not
  // return the stale id (its spans would land on a series the host no
  // longer tracks and vanish from the export)
  const reqs = mixedRequests().concat(eventRequests()).map((r) => otlp.encodeTraces(r));
  for (const [cfg, collide, batched] of [[{ resource_metrics_cache_size: 1 }, false, false],
    [{ resource_metrics_cache_size: 2 }, true, false], [{}, true, true], [{ resource_metrics_cache_size: 1 }, false, true],
    [{ resource_metrics_cache_size: 1, dimensions: [{ name: 'k8s.pod.name' }] }, true, true]]) {
    const out = [];
    for (const native of [true, false]) {
      const addon = native ? new NativeColumnizerFakeAddon() : new FakeAddon();
      addon.collide = collide;
      addon.batched = batched;
      const t = { now: 1000n };
      const conn = new SpanMetricsConnector(Object.assign({ batch_size: 16, columnizer_threads: 4 }, cfg),
        { addon, rules: DEMO_SPAN_NAME_RULES, native, clock: () => (t.now += 1n) });
      const real = keys.seriesHashSeeded;
      if (collide) keys.seriesHashSeeded = (rh, k, seed) => (seed === 0n ? 42n : real(rh, k, seed));
      const exports = [];
      try {
        const errs = conn.consumeTracesBatch(reqs.slice(0, 8));
        assert.ok(errs.every((e) => e === null));
        exports.push(otlp.encodeMetrics(conn.exportMetrics()).toString('hex'));
        for (const r of reqs) conn.consumeTraces(r);  // one request at a time (the T <= 1 path)
        exports.push(otlp.encodeMetrics(conn.exportMetrics()).toString('hex'));
        assert.ok(conn.consumeTracesBatch(reqs.slice(3, 12)).every((e) => e === null));
        for (const r of reqs.slice(0, 5)) conn.consumeTraces(r);
        exports.push(otlp.encodeMetrics(conn.exportMetrics()).toString('hex'));
      } finally {
        keys.seriesHashSeeded = real;
      }
      if (native) assert.ok(conn.stats().nativeRequests > 0 && conn.stats().jsRequests === 0);
      out.push(exports);
    }
    assert.deepStrictEqual(out[0], out[1], JSON.stringify([cfg, collide]));
  }
});

test('pipeline queue: requests of one event-loop turn go through consumeTracesBatch', async () => {
  const addon = new NativeColumnizerFakeAddon();
  let batches = 0;
  const real = addon.columnizeBatch.bind(addon);
  addon.columnizeBatch = (c, bufs) => { batches += 1; return real(c, bufs); };
  const { TracesToMetricsPipeline: P } = require(path.join(lib, 'pipeline'));
  const p = new P({ addon, receiver: false, exporter: false, memoryLimiter: false, spanmetrics: { columnizer_threads: 2 } });
  const good = otlp.encodeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('y')]]]));
  const res = await Promise.allSettled([p.consumeTracesQueued(good), p.consumeTracesQueued(good.subarray(0, 9)),
    p.consumeTracesQueued(good)]);
  assert.deepStrictEqual(res.map((r) => r.status), ['fulfilled', 'rejected', 'fulfilled']);
  assert.strictEqual(batches, 1);
  const calls = dpsOf(p.connector.exportMetrics(), 'traces.span.metrics.calls');
  assert.deepStrictEqual(calls.map((d) => d.asInt), [2n, 2n]);
  p.connector.shutdown();
});

test('pipeline constructor (README / INTEGRATION demo path) applies the demo transform rules', () => {
  const { TracesToMetricsPipeline: P } = require(path.join(lib, 'pipeline'));
  const p = new P({ addon: new FakeAddon(), receiver: false, exporter: false, memoryLimiter: false });
  assert.deepStrictEqual(p.rules, DEMO_SPAN_NAME_RULES);
  p.consumeTraces(otlp.encodeTraces(request([[{ 'service.name': 'frontend' }, [
    span('GET /api/products/0PUK6V6EV0?currency=USD'), span('GET /api/products/66VCHSJNUP'),
    span('GET /api/cart?sessionId=1')]]])));
  const names = dpsOf(p.connector.exportMetrics(), 'traces.span.metrics.calls')
    .map((d) => d.attributes.find((a) => a.key === 'span.name').value.value).sort();
  assert.deepStrictEqual(names, ['GET /api/cart', 'GET /api/products/{productId}']);
  p.connector.shutdown();
  const none = new P({ addon: new FakeAddon(), receiver: false, exporter: false, memoryLimiter: false, transform: [] });
  assert.deepStrictEqual(none.rules, []);
  none.connector.shutdown();
});

test('consumeTracesBatch: a failure part-way rejects only the requests not yet applied', () => {
  const addon = new NativeColumnizerFakeAddon();
  let drains = 0;
  addon.columnizerIngest = (c) => {  // the engine fails on its second batch of columns
    drains += 1;
    // a failing ingest that leaves the columns buffered (the worst case: the
    // connector itself must drop them, advisor r3)
    if (drains === 2) throw new Error('SA_EDEVICE: device lost');
    const b = addon.real.columnizerTake(c);
    addon.ingest(null, b);
    return b.keyHash.length;
  };
  const conn = new SpanMetricsConnector({ batch_size: 4, columnizer_threads: 1 }, { addon, rules: DEMO_SPAN_NAME_RULES });
  const req = (k) => otlp.encodeTraces(request([[{ 'service.name': `s${k}` }, [span('a'), span('b'), span('c')]]]));
  // one drain per batch here (6 spans >= 4); the second batch's drain fails:
  // its requests (whose spans were in the failed columns) are rejected, the
  // first batch's stay acknowledged
  assert.deepStrictEqual(conn.consumeTracesBatch([req(0), req(1)]), [null, null]);
  const errs = conn.consumeTracesBatch([req(2), req(3)]);
  assert.ok(errs.every((e) => e instanceof Error && e.deferred === true), String(errs));
  // the senders retry the rejected requests: each span counts once
  assert.deepStrictEqual(conn.consumeTracesBatch([req(2), req(3)]), [null, null]);
  const calls = dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls');
  assert.strictEqual(calls.length, 12);  // 4 services x 3 span names
  assert.ok(calls.every((d) => Number(d.asInt) === 1), calls.map((d) => String(d.asInt)).join(","));
  const addon2 = new NativeColumnizerFakeAddon();
  addon2.columnizeBatch = () => { throw new Error('columnizer broke'); };
  const c2 = new SpanMetricsConnector({ columnizer_threads: 2 }, { addon: addon2, rules: DEMO_SPAN_NAME_RULES });
  const e2 = c2.consumeTracesBatch([req(0), req(1)]);
  assert.ok(e2.every((e) => e instanceof Error && /columnizer broke/.test(e.message)));
  conn.shutdown();
  c2.shutdown();
});

test('native columnizer: invalid UTF-8 falls back to JavaScript; malformed bytes are rejected', () => {
  const addon = new NativeColumnizerFakeAddon();
  const conn = new SpanMetricsConnector({}, { addon, rules: DEMO_SPAN_NAME_RULES });
  const body = otlp.encodeTraces(request([[{ 'service.name': 'a' }, [span('GET /x\u00e9')]]]));
  const bad = Buffer.from(body);
  bad[bad.indexOf(0xC3)] = 0xFF;  // break the UTF-8 of the span name
  conn.consumeTraces(bad);
  assert.strictEqual(conn.stats().jsRequests, 1);
  conn.consumeTraces(body);
  assert.strictEqual(conn.stats().nativeRequests, 1);
  assert.throws(() => conn.consumeTraces(body.subarray(0, body.length - 2)), /OTLP request|truncated/);
  const c = dpsOf(conn.exportMetrics(), 'traces.span.metrics.calls');
  assert.strictEqual(c.length, 2);
});

test('native building blocks: xxh64 and Go FormatFloat agree with the JavaScript ones', () => {
  const real = require('../lib/addon').load();
  const { xxh64 } = require(path.join(lib, 'xxh64'));
  for (let n = 0; n < 80; n++) {
    const b = Uint8Array.from({ length: n }, (_, i) => (i * 31 + n) & 255);
    assert.strictEqual(real.columnizerSelfTest('xxh64', b, 0n), xxh64(Buffer.from(b), 0n));
    assert.strictEqual(real.columnizerSelfTest('xxh64', b, 1n), xxh64(Buffer.from(b), 1n));
  }
  const xs = [0, -0, 1, -1, 0.1, 1 / 3, 1e21, 1e-7, 1.5e-7, 123456789.125, 2 ** 53, 5e-324, 1.7976931348623157e308,
    NaN, Infinity, -Infinity, 1e22, 123e-20, 0.000001, 1e-6];
  for (const x of xs) assert.strictEqual(real.columnizerSelfTest('formatFloat', x), keys.formatFloat(x), String(x));
});

// ------------------------------------------------- receiver / exporter / pipeline
const http = require('http');
const http2 = require('http2');
const zlib = require('zlib');
const { OtlpReceiver, MemoryLimiter, grpcFrame, grpcUnframe, TRACE_EXPORT_PATH } = require(path.join(lib, 'receiver'));
const { TracesToMetricsPipeline } = require(path.join(lib, 'pipeline'));

function post(port, pathName, body, headers) {
  return new Promise((resolve, reject) => {
    const req = http.request({ host: '127.0.0.1', port, path: pathName, method: 'POST', headers }, (res) => {
      const chunks = [];
      res.on('data', (c) => chunks.push(c));
      res.on('end', () => resolve({ status: res.statusCode, body: Buffer.concat(chunks) }));
    });
    req.on('error', reject);
    req.end(body);
  });
}

function grpcCall(port, pathName, frames, extra = {}) {
  return new Promise((resolve, reject) => {
    const client = http2.connect(`http://127.0.0.1:${port}`);
    client.on('error', reject);
    const req = client.request(Object.assign({ ':method': 'POST', ':path': pathName,
      'content-type': 'application/grpc', te: 'trailers' }, extra));
    const chunks = [];
    let trailers = {};
    req.on('trailers', (t) => { trailers = t; });
    req.on('data', (c) => chunks.push(c));
    req.on('end', () => { client.close(); resolve({ body: Buffer.concat(chunks), trailers }); });
    req.on('error', reject);
    req.end(frames);
  });
}

test('receiver: OTLP/HTTP and OTLP/gRPC deliver request bytes; errors map to retryable codes', async () => {
  const got = [];
  let refuse = false;
  const rx = await new OtlpReceiver({ httpPort: 0, grpcPort: 0, onTraces: (b) => {
    if (refuse) { const e = new Error('full'); e.refused = true; throw e; }
    got.push(otlp.decodeTraces(b));
  } }).start();
  try {
    const body = otlp.encodeTraces(request([[{ 'service.name': 'a' }, [span('x'), span('y')]]]));
    let r = await post(rx.httpPort, '/v1/traces', body, { 'Content-Type': 'application/x-protobuf' });
    assert.strictEqual(r.status, 200);
    r = await post(rx.httpPort, '/v1/traces', zlib.gzipSync(body),
      { 'Content-Type': 'application/x-protobuf', 'Content-Encoding': 'gzip' });
    assert.strictEqual(r.status, 200);
    r = await post(rx.httpPort, '/v1/traces', Buffer.from('{}'), { 'Content-Type': 'application/json' });
    assert.strictEqual(r.status, 415);
    r = await post(rx.httpPort, '/v1/metrics', body, { 'Content-Type': 'application/x-protobuf' });
    assert.strictEqual(r.status, 404);
    let g = await grpcCall(rx.grpcPort, TRACE_EXPORT_PATH, Buffer.concat([grpcFrame(body), grpcFrame(body)]));
    assert.strictEqual(g.trailers['grpc-status'], '0');
    assert.deepStrictEqual(grpcUnframe(g.body), [Buffer.alloc(0)]);
    const gz = zlib.gzipSync(body);
    const cf = grpcFrame(gz);
    cf[0] = 1;  // compressed flag
    g = await grpcCall(rx.grpcPort, TRACE_EXPORT_PATH, cf, { 'grpc-encoding': 'gzip' });
    assert.strictEqual(g.trailers['grpc-status'], '0');
    assert.strictEqual(got.length, 5);
    assert.strictEqual(got[4].resourceSpans[0].scopeSpans[0].spans[1].name, 'y');
    g = await grpcCall(rx.grpcPort, '/x.Y/Z', grpcFrame(body));
    assert.strictEqual(g.trailers['grpc-status'], '12');
    refuse = true;
    r = await post(rx.httpPort, '/v1/traces', body, { 'Content-Type': 'application/x-protobuf' });
    assert.strictEqual(r.status, 503);
    g = await grpcCall(rx.grpcPort, TRACE_EXPORT_PATH, grpcFrame(body));
    assert.strictEqual(g.trailers['grpc-status'], '14');
  } finally {
    await rx.close();
  }
});

test('memory_limiter: refuses above the soft limit, recovers below it', () => {
  let rss = 10;
  const m = new MemoryLimiter({ limit_mib: 100, spike_limit_mib: 20, check_interval_ms: 0, usage: () => rss * 1048576 });
  m.check();
  rss = 81;
  assert.throws(() => m.check(), (e) => e.refused === true);
  rss = 79;
  m.check();
  assert.strictEqual(m.refused, 1);
  const demo = new MemoryLimiter({ total: 1000, usage: () => 0 });
  assert.strictEqual(demo.limit, 800);
  assert.strictEqual(demo.soft, 550);
});

test('pipeline: OTLP/HTTP in -> transform -> connector -> otlphttp out', async () => {
  const posted = [];
  const sink = http.createServer((req, res) => {
    const chunks = [];
    req.on('data', (c) => chunks.push(c));
    req.on('end', () => { posted.push({ url: req.url, type: req.headers['content-type'], body: Buffer.concat(chunks) }); res.end(); });
  });
  await new Promise((r) => sink.listen(0, '127.0.0.1', r));
  // a collector config in the demo's shape (otelcol-config.yml:100-127): the
  // transform rules and wiring come from it
  const p = await TracesToMetricsPipeline.fromCollectorConfig(DEMO_LIKE_CONFIG, { addon: new FakeAddon(),
    clock: () => 7n, receiver: { httpPort: 0, grpcPort: 0 }, memoryLimiter: { limit_mib: 1e9 },
    exporter: { endpoint: `http://127.0.0.1:${sink.address().port}/api/v1/otlp` } }).start();
  try {
    const body = otlp.encodeTraces(request([[{ 'service.name': 'frontend' }, [
      span('GET /api/products/ABC?currency=USD'), span('GET /api/products/XYZ')]]]));
    const r = await post(p.receiver.httpPort, '/v1/traces', body, { 'Content-Type': 'application/x-protobuf' });
    assert.strictEqual(r.status, 200);
    await p.flush();
    assert.strictEqual(posted.length, 1);
    assert.strictEqual(posted[0].url, '/api/v1/otlp/v1/metrics');
    assert.strictEqual(posted[0].type, 'application/x-protobuf');
    const m = otlp.decodeMetrics(posted[0].body);
    const calls = m.resourceMetrics[0].scopeMetrics[0].metrics[0].sum.dataPoints;
    assert.strictEqual(calls.length, 1);  // both names collapse to one series (A12)
    assert.strictEqual(calls[0].asInt, 2n);
    assert.strictEqual(attr(calls[0], 'span.name').value, 'GET /api/products/{productId}');
  } finally {
    await p.shutdown();
    await new Promise((r) => sink.close(r));
  }
});


// An ExportTraceServiceRequest whose one resource attribute is an array
// nested `levels` deep, written back to front in one buffer (no recursion).
function deepNestedRequest(levels) {
  const varintLen = (n) => { let l = 1; while (n >= 128) { n = Math.floor(n / 128); l++; } return l; };
  const inner = Buffer.from([0x0a, 0x01, 0x78]);  // AnyValue{string_value: "x"}
  let size = inner.length;
  const sizes = [];
  for (let i = 0; i < levels; i++) {  // ArrayValue{values: any} then AnyValue{array_value: arr}
    const arr = 1 + varintLen(size) + size;
    const any = 1 + varintLen(arr) + arr;
    sizes.push([size, arr]);
    size = any;
  }
  const buf = Buffer.alloc(size);
  let p = size - inner.length;
  inner.copy(buf, p);
  const putVarint = (n) => {  // ending at p
    const bytes = [];
    do { let b = n % 128; n = Math.floor(n / 128); if (n) b |= 128; bytes.push(b); } while (n);
    p -= bytes.length;
    Buffer.from(bytes).copy(buf, p);
  };
  for (let i = 0; i < levels; i++) {  // innermost level first: the buffer fills back to front
    const [inSize, arr] = sizes[i];
    putVarint(inSize); buf[--p] = 0x0a;   // ArrayValue.values (1, LEN)
    putVarint(arr); buf[--p] = 0x2a;      // AnyValue.array_value (5, LEN)
  }
  const w = (field, payload) => Buffer.concat([Buffer.from([(field << 3) | 2]), varintBuf(payload.length), payload]);
  const varintBuf = (n) => { const b = []; do { let x = n % 128; n = Math.floor(n / 128); if (n) x |= 128; b.push(x); } while (n); return Buffer.from(b); };
  const kv = (key, anyBytes) => Buffer.concat([w(1, Buffer.from(key)), w(2, anyBytes)]);
  const resource = Buffer.concat([w(1, kv('service.name', Buffer.from([0x0a, 0x01, 0x61]))), w(1, kv('deep', buf))]);
  const spanBytes = Buffer.concat([w(1, Buffer.alloc(16, 1)), w(5, Buffer.from('op'))]);
  const rs = Buffer.concat([w(1, resource), w(2, w(2, spanBytes))]);
  return w(1, rs);
}

test('receiver: an attribute nested 100k levels deep is a 400, and the host keeps serving', async () => {
  const body = deepNestedRequest(100000);
  for (const addon of [new NativeColumnizerFakeAddon(), new FakeAddon()]) {
    const p = await new TracesToMetricsPipeline({ addon, clock: () => 7n, exporter: false, memoryLimiter: false,
      receiver: { httpPort: 0, grpcPort: 0 } }).start();
    try {
      let r = await post(p.receiver.httpPort, '/v1/traces', body, { 'Content-Type': 'application/x-protobuf' });
      assert.strictEqual(r.status, 400, String(r.body));
      const g = await grpcCall(p.receiver.grpcPort, TRACE_EXPORT_PATH, grpcFrame(body));
      assert.strictEqual(g.trailers['grpc-status'], '3');
      const ok = otlp.encodeTraces(request([[{ 'service.name': 'a' }, [span('x')]]]));
      r = await post(p.receiver.httpPort, '/v1/traces', ok, { 'Content-Type': 'application/x-protobuf' });
      assert.strictEqual(r.status, 200);
      // 100 levels is still a valid request
      r = await post(p.receiver.httpPort, '/v1/traces', deepNestedRequest(99), { 'Content-Type': 'application/x-protobuf' });
      assert.strictEqual(r.status, 200, String(r.body));
    } finally {
      await p.shutdown();
    }
  }
});

test('receiver: the body limit applies after decompression (gzip bomb -> 413 / RESOURCE_EXHAUSTED)', async () => {
  const seen = [];
  const rx = await new OtlpReceiver({ httpPort: 0, grpcPort: 0, maxBodyBytes: 1 << 20,
    onTraces: (b) => seen.push(b.length) }).start();
  try {
    const bomb = zlib.gzipSync(Buffer.alloc(64 << 20));  // 64 MiB of zeros in ~64 KiB
    assert.ok(bomb.length < 1 << 20);
    let r = await post(rx.httpPort, '/v1/traces', bomb,
      { 'Content-Type': 'application/x-protobuf', 'Content-Encoding': 'gzip' });
    assert.strictEqual(r.status, 413);
    const frame = Buffer.concat([Buffer.from([1, 0, 0, 0, 0]), bomb]);
    frame.writeUInt32BE(bomb.length, 1);
    const g = await grpcCall(rx.grpcPort, TRACE_EXPORT_PATH, frame, { 'grpc-encoding': 'gzip' });
    assert.strictEqual(g.trailers['grpc-status'], '8');
    r = await post(rx.httpPort, '/v1/traces', Buffer.from('not gzip'),
      { 'Content-Type': 'application/x-protobuf', 'Content-Encoding': 'gzip' });
    assert.strictEqual(r.status, 400);
    assert.deepStrictEqual(seen, []);
  } finally {
    await rx.close();
  }
});

// ------------------------------------------------------------- collector config (YAML + OTTL)
const cc = require(path.join(lib, 'collector_config'));
const DEMO_LIKE_CONFIG = [
  'processors:',
  '  batch:',
  '  memory_limiter:',
  '    check_interval: 5s',
  '    limit_percentage: 80',
  '  transform:',
  '    error_mode: ignore',
  '    trace_statements:',
  '      - context: span',
  '        statements:',
  '          # a comment between items',
  '          - replace_pattern(name, "\\\\?.*", "")',
  '          - replace_match(name, "GET /api/products/*", "GET /api/products/{productId}")',
  'connectors:',
  '  spanmetrics:',
  'service:',
  '  pipelines:',
  '    traces:',
  '      receivers: [otlp]',
  '      processors: [memory_limiter, transform, batch]',
  '      exporters: [otlp, debug, spanmetrics]',
  '    metrics:',
  '      receivers: [otlp, spanmetrics]',
  '      exporters: [otlphttp/prometheus]',
].join('\n');

test('yaml: mappings, sequences, scalars, flow values, comments', () => {
  const v = cc.parseYaml([
    'a: 1', 'b: "x\\ty"  # trailing comment', "c: 'it''s'", 'd:', 'e: [1, two, "3"]',
    'f: {k: v, n: 2}', 'g:', '  - x', '  - k: 1', '    j: true', '  -', '    - nested',
    'h:', '- same-indent item', 'i: http://host:4318/path#frag', 'j: ~', 'k: 1.5e3', 'l: 5s',
  ].join('\n'));
  assert.deepStrictEqual(v, { a: 1, b: 'x\ty', c: "it's", d: null, e: [1, 'two', '3'], f: { k: 'v', n: 2 },
    g: ['x', { k: 1, j: true }, ['nested']], h: ['same-indent item'], i: 'http://host:4318/path#frag',
    j: null, k: 1500, l: '5s' });
  assert.throws(() => cc.parseYaml('a: 1\n   b: 2'), cc.YamlError);
  assert.throws(() => cc.parseYaml('a: "open'), cc.YamlError);
});

test('yaml: env expansion and the multi-file deep merge of --config flags', () => {
  const cfg = cc.loadCollectorConfig(['x:\n  ep: ${env:HOST}:${PORT}\n  keep: 1\nl: [a]',
    'x:\n  add: 2\nl: [b]'], { HOST: 'h', PORT: '9' });
  assert.deepStrictEqual(cfg, { x: { ep: 'h:9', keep: 1, add: 2 }, l: ['b'] });
});

test('collector config: spanmetrics block, transform rules and wiring of the demo shape', () => {
  const o = cc.pipelineOptions(cc.loadCollectorConfig([DEMO_LIKE_CONFIG], {}));
  assert.deepStrictEqual(o.spanmetrics, {});
  assert.deepStrictEqual(o.memoryLimiter, { check_interval: '5s', limit_percentage: 80 });
  assert.deepStrictEqual(o.wiring.traces.processors, ['memory_limiter', 'transform', 'batch']);
  assert.strictEqual(o.transform.length, 2);
  assert.strictEqual(o.transform.errorMode, 'ignore');
  for (const [a, b] of [['GET /api/products/0PUK6V6EV0?x=1', 'GET /api/products/{productId}'],
    ['GET /api/cart?sessionId=1', 'GET /api/cart'], ['POST /api/products/1', 'POST /api/products/1']])
    assert.strictEqual(applyRules(a, o.transform), b);
  // the rules keep their native descriptors, so the C++ columnizer can run them
  assert.deepStrictEqual(o.transform.map((r) => r.native.kind), ['strip_query', 'glob']);
});

test('collector config: unsupported statements and broken wiring are configuration errors', () => {
  const mk = (stmt) => cc.loadCollectorConfig([DEMO_LIKE_CONFIG.replace(
    'replace_pattern(name, "\\\\?.*", "")', stmt)], {});
  assert.throws(() => cc.pipelineOptions(mk('set(attributes["x"], "y")')), cc.ConfigError);
  assert.throws(() => cc.pipelineOptions(mk('replace_pattern(name, "a", "b") where kind == 1')), cc.ConfigError);
  assert.throws(() => cc.pipelineOptions(cc.loadCollectorConfig([DEMO_LIKE_CONFIG.replace(
    'exporters: [otlp, debug, spanmetrics]', 'exporters: [otlp]')], {})), cc.ConfigError);
  assert.throws(() => cc.spanmetricsConfig({ connectors: {} }), cc.ConfigError);
  // explicit buckets and dimensions pass through to the connector config
  const o = cc.pipelineOptions(cc.loadCollectorConfig([DEMO_LIKE_CONFIG.replace('  spanmetrics:',
    '  spanmetrics:\n    histogram:\n      explicit:\n        buckets: [2ms, 4ms, 1s]\n' +
    '    dimensions:\n      - name: http.method\n        default: GET')], {}));
  assert.deepStrictEqual(o.spanmetrics, { histogram: { explicit: { buckets: ['2ms', '4ms', '1s'] } },
    dimensions: [{ name: 'http.method', default: 'GET' }] });
});

// ------------------------------------------------------------------ runner
(async () => {
  let failed = 0;
  for (const t of tests) {
    try {
      await t.fn();
      console.log(`ok   ${t.name}`);
    } catch (e) {
      failed += 1;
      console.log(`FAIL ${t.name}\n${e.stack}`);
      break;
    }
  }
  console.log(`${tests.length - failed}/${tests.length} passed`);
  process.exit(failed ? 1 : 0);
})();
