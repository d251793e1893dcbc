'use strict';
/**
 * Test bridge for tests/test_node_host.py: reads one JSON command on stdin,
 * writes one JSON result on stdout.  Typed attribute values travel as
 * [type, payload]: ["string", s] | ["bool", b] | ["int", "decimal"] |
 * ["double", x] | ["bytes", "hex"] | ["array", [typed...]] |
 * ["kvlist", [[key, typed]...]] | ["empty", null].
 *
 *   {"cmd": "keys", "vectors": [...]}            key strings, resource and series hashes
 *   {"cmd": "decode_traces", "b64": "..."}      decoded request (u64 as decimal strings)
 *   {"cmd": "encode_traces", "req": {...}}      -> {"b64": ...}
 *   {"cmd": "encode_metrics", "req": {...}}     -> {"b64": ...}
 *   {"cmd": "xxh64", "cases": [[hex, seed]...]} -> hex digests
 *   {"cmd": "transform", "names": [...]}        demo transform rules applied
 *   {"cmd": "collector_config", "texts": [yaml...], "env": {...}, "names": [...]}
 *        -> the pipeline options a collector config yields (lib/collector_config.js):
 *           spanmetrics block, memory limiter, wiring, and `names` through the
 *           transform rules it declares
 *   {"cmd": "connector_export", "requests": [b64...], "texts": [yaml...]?, "spanmetrics": {...}?}
 *        -> {"b64": ExportMetricsServiceRequest} from a TracesToMetricsPipeline over
 *           the test stand-in addon (host logic only: names, attributes, layout)
 */
const path = require('path');
const lib = path.join(__dirname, '..', 'lib');
const otlp = require(path.join(lib, 'otlp'));
const keys = require(path.join(lib, 'keys'));
const { xxh64 } = require(path.join(lib, 'xxh64'));
const { applyRules, DEMO_SPAN_NAME_RULES } = require(path.join(lib, 'transform'));
const collectorConfig = require(path.join(lib, 'collector_config'));
const { TracesToMetricsPipeline } = require(path.join(lib, 'pipeline'));
const { FakeAddon } = require('./fake_addon');

function fromTyped([t, v]) {
  switch (t) {
    case 'string': return { type: 'string', value: v };
    case 'bool': return { type: 'bool', value: !!v };
    case 'int': return { type: 'int', value: BigInt(v) };
    case 'double': return { type: 'double', value: v === 'nan' ? NaN : v === 'inf' ? Infinity : v === '-inf' ? -Infinity : v };
    case 'bytes': return { type: 'bytes', value: Uint8Array.from(Buffer.from(v, 'hex')) };
    case 'array': return { type: 'array', value: v.map(fromTyped) };
    case 'kvlist': return { type: 'kvlist', value: v.map(([key, x]) => ({ key, value: fromTyped(x) })) };
    default: return { type: 'empty', value: null };
  }
}

function toTyped(v) {
  switch (v.type) {
    case 'string': return ['string', v.value];
    case 'bool': return ['bool', v.value];
    case 'int': return ['int', v.value.toString()];
    case 'double': return ['double', Number.isFinite(v.value) ? v.value : String(v.value)];
    case 'bytes': return ['bytes', Buffer.from(v.value).toString('hex')];
    case 'array': return ['array', v.value.map(toTyped)];
    case 'kvlist': return ['kvlist', v.value.map((kv) => [kv.key, toTyped(kv.value)])];
    default: return ['empty', null];
  }
}

const kvsFrom = (obj) => (obj || []).map(([key, v]) => ({ key, value: fromTyped(v) }));
const kvsTo = (kvs) => kvs.map((kv) => [kv.key, toTyped(kv.value)]);
const hex = (b) => Buffer.from(b).toString('hex');
const u64hex = (x) => x.toString(16).padStart(16, '0');

function reqFromJson(req) {
  return { resourceSpans: req.resource_spans.map((rs) => ({
    resource: { attributes: kvsFrom(rs.resource) },
    scopeSpans: rs.scope_spans.map((ss) => ({ scope: { name: ss.scope || '' },
      spans: ss.spans.map((s) => ({ traceId: Uint8Array.from(Buffer.from(s.trace_id, 'hex')),
        spanId: Uint8Array.from(Buffer.from(s.span_id || '', 'hex')), name: s.name, kind: s.kind,
        startTimeUnixNano: BigInt(s.start), endTimeUnixNano: BigInt(s.end),
        attributes: kvsFrom(s.attributes), status: { code: s.status || 0, message: s.message || '' } })) })) })) };
}

function reqToJson(req) {
  return { resource_spans: req.resourceSpans.map((rs) => ({ resource: kvsTo(rs.resource.attributes),
    scope_spans: rs.scopeSpans.map((ss) => ({ scope: ss.scope.name, spans: ss.spans.map((s) => ({
      trace_id: hex(s.traceId), span_id: hex(s.spanId), name: s.name, kind: s.kind,
      start: s.startTimeUnixNano.toString(), end: s.endTimeUnixNano.toString(),
      attributes: kvsTo(s.attributes), status: s.status.code, message: s.status.message })) })) })) };
}

function metricsFromJson(req) {
  const dp = (p) => Object.assign({}, p, {
    attributes: kvsFrom(p.attributes),
    startTimeUnixNano: BigInt(p.start || 0), timeUnixNano: BigInt(p.time || 0),
    count: p.count !== undefined ? BigInt(p.count) : undefined,
    asInt: p.as_int !== undefined ? BigInt(p.as_int) : undefined,
    asDouble: p.as_double,
    bucketCounts: p.bucket_counts ? p.bucket_counts.map(BigInt) : undefined,
    explicitBounds: p.explicit_bounds });
  return { resourceMetrics: req.resource_metrics.map((rm) => ({ resource: { attributes: kvsFrom(rm.resource) },
    scopeMetrics: [{ scope: { name: rm.scope }, metrics: rm.metrics.map((m) => {
      const out = { name: m.name, unit: m.unit || '', description: m.description || '' };
      if (m.kind === 'sum') out.sum = { dataPoints: m.points.map(dp), aggregationTemporality: m.temporality, isMonotonic: m.monotonic };
      else if (m.kind === 'histogram') out.histogram = { dataPoints: m.points.map(dp), aggregationTemporality: m.temporality };
      else out.gauge = { dataPoints: m.points.map(dp) };
      return out;
    }) }] })) };
}

function run(cmd) {
  switch (cmd.cmd) {
    case 'keys':
      return cmd.vectors.map((v) => {
        const span = new Map(kvsFrom(v.span_attrs).map((kv) => [kv.key, kv.value]));
        const res = new Map(kvsFrom(v.resource_attrs).map((kv) => [kv.key, kv.value]));
        const key = keys.buildKey(v.service, v.span_name, v.kind, v.status, v.dims || [], span, res,
          new Set(v.exclude || []));
        const rh = keys.resourceHash(res);
        return { key: hex(key), resource_hash: u64hex(rh), series: u64hex(keys.seriesHash(rh, key)),
          attrs: kvsTo(keys.buildAttributes(v.service, v.span_name, v.kind, v.status, v.dims || [], span, res,
            new Set(v.exclude || []))) };
      });
    case 'decode_traces': return reqToJson(otlp.decodeTraces(Buffer.from(cmd.b64, 'base64')));
    case 'encode_traces': return { b64: otlp.encodeTraces(reqFromJson(cmd.req)).toString('base64') };
    case 'encode_metrics': return { b64: otlp.encodeMetrics(metricsFromJson(cmd.req)).toString('base64') };
    case 'xxh64': return cmd.cases.map(([h, seed]) => u64hex(xxh64(Buffer.from(h, 'hex'), BigInt(seed))));
    case 'transform': return cmd.names.map((n) => applyRules(n, DEMO_SPAN_NAME_RULES));
    case 'collector_config': {
      const cfg = collectorConfig.loadCollectorConfig(cmd.texts, cmd.env || {});
      const o = collectorConfig.pipelineOptions(cfg);
      return { spanmetrics: o.spanmetrics, memory_limiter: o.memoryLimiter, wiring: o.wiring,
        n_rules: o.transform.length, error_mode: o.transform.errorMode || null,
        names: (cmd.names || []).map((n) => applyRules(n, o.transform)) };
    }
    case 'connector_export': {
      const common = { addon: new FakeAddon(), receiver: false, exporter: false, native: false,
        clock: () => 1700000000000000000n };
      const p = cmd.texts
        ? TracesToMetricsPipeline.fromCollectorConfig(cmd.texts, Object.assign(common, { env: {},
          spanmetrics: cmd.spanmetrics || {} }))
        : new TracesToMetricsPipeline(Object.assign(common, { spanmetrics: cmd.spanmetrics || {} }));
      for (const r of cmd.requests) p.consumeTraces(Buffer.from(r, 'base64'));
      return p.flush().then((bytes) => ({ b64: Buffer.from(bytes).toString('base64') }));
    }
    default: throw new Error(`unknown cmd ${cmd.cmd}`);
  }
}

let input = '';
process.stdin.setEncoding('utf8');
process.stdin.on('data', (c) => { input += c; });
process.stdin.on('end', () => {
  Promise.resolve(run(JSON.parse(input))).then((out) => process.stdout.write(JSON.stringify(out)),
    (e) => { process.stderr.write(String(e && e.stack || e)); process.exit(1); });
});
