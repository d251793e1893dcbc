'use strict';
/**
 * Series identity on the host (the device sees only u64 ids) -- the Node
 * mirror of opentelemetry-demo_amd/spanagg/keys.py, restating the connector's
 * key building ([UPSTREAM] spanmetricsconnector connector.go buildKey +
 * concatDimensionValue, buildAttributes; traceutil.SpanKindStr /
 * StatusCodeStr; SURVEY.md rows a6-a8 and A5-A7):
 *
 *   key = service.name \0 span.name \0 SpanKindStr \0 StatusCodeStr [\0 dim]*
 *
 * Attribute values are decoded OTLP AnyValues: {type, value} with type one of
 * 'string' | 'bool' | 'int' (BigInt) | 'double' | 'bytes' (Uint8Array) |
 * 'array' (AnyValue[]) | 'kvlist' ({key, value}[]) | 'empty'.
 */
const xxh64js = require('./xxh64').xxh64;

// The addon's native xxh64 once addon.js has loaded it (same function: the
// addon's self-test checks the two against each other); the JavaScript BigInt
// restatement stays for hosts without the addon (the fake-addon tests).
let xxh64 = xxh64js;
function useNativeXxh64(fn) { xxh64 = fn || xxh64js; }

const SPAN_KIND_STR = ['SPAN_KIND_UNSPECIFIED', 'SPAN_KIND_INTERNAL', 'SPAN_KIND_SERVER',
  'SPAN_KIND_CLIENT', 'SPAN_KIND_PRODUCER', 'SPAN_KIND_CONSUMER'];
const STATUS_CODE_STR = ['STATUS_CODE_UNSET', 'STATUS_CODE_OK', 'STATUS_CODE_ERROR'];
const SERVICE_NAME_KEY = 'service.name';
const SPAN_NAME_KEY = 'span.name';
const SPAN_KIND_KEY = 'span.kind';
const STATUS_CODE_KEY = 'status.code';

/** traceutil.SpanKindStr: out-of-range -> "" (A7). */
const spanKindStr = (k) => (k >= 0 && k < SPAN_KIND_STR.length ? SPAN_KIND_STR[k] : '');
/** traceutil.StatusCodeStr: out-of-range -> "" (A7). */
const statusCodeStr = (c) => (c >= 0 && c < STATUS_CODE_STR.length ? STATUS_CODE_STR[c] : '');

/** Go strconv.FormatFloat(f, 'f', -1, 64): shortest round-trip digits, positional. */
function formatFloat(f) {
  if (Number.isNaN(f)) return 'NaN';
  if (f === Infinity) return '+Inf';
  if (f === -Infinity) return '-Inf';
  if (Object.is(f, -0)) return '-0';
  const s = String(f);  // shortest round-trip, maybe with an exponent
  const m = /^(-?)(\d)(?:\.(\d+))?e([+-]\d+)$/.exec(s);
  if (!m) return s;
  const [, sign, d0, frac = '', e] = m;
  const exp = parseInt(e, 10);
  const digits = d0 + frac;
  if (exp >= 0) {
    return sign + (exp + 1 >= digits.length ? digits + '0'.repeat(exp + 1 - digits.length)
      : digits.slice(0, exp + 1) + '.' + digits.slice(exp + 1));
  }
  return sign + '0.' + '0'.repeat(-exp - 1) + digits;
}

function rawJson(v) {  // AsString() of slices and maps is the JSON of their raw values
  switch (v.type) {
    case 'string': return JSON.stringify(v.value);
    case 'bool': return v.value ? 'true' : 'false';
    case 'int': return v.value.toString();
    case 'double': return Number.isFinite(v.value) ? String(v.value) : JSON.stringify(formatFloat(v.value));
    case 'bytes': return JSON.stringify(Buffer.from(v.value).toString('base64'));
    case 'array': return '[' + v.value.map(rawJson).join(',') + ']';
    case 'kvlist': return '{' + v.value.map((kv) => JSON.stringify(kv.key) + ':' + rawJson(kv.value)).join(',') + '}';
    default: return 'null';
  }
}

/** pcommon.Value.AsString() for decoded OTLP values. */
function asString(v) {
  if (v === undefined || v === null) return '';
  switch (v.type) {
    case 'string': return v.value;
    case 'bool': return v.value ? 'true' : 'false';
    case 'int': return v.value.toString();
    case 'double': return formatFloat(v.value);
    case 'bytes': return Buffer.from(v.value).toString('base64');
    case 'array': case 'kvlist': return rawJson(v);
    default: return '';
  }
}

/** Python type tag of the value kind (keys.py resource_hash uses type(v).__name__). */
const TYPE_TAG = { string: 'str', bool: 'bool', int: 'int', double: 'float', bytes: 'bytes',
  array: 'list', kvlist: 'dict', empty: 'NoneType' };

/** attrs: [{key, value}] -> Map key -> value (last wins, as pcommon.Map.PutX would keep one). */
function attrMap(attrs) {
  const m = new Map();
  for (const kv of attrs || []) m.set(kv.key, kv.value);
  return m;
}

/**
 * buildKey.  dims = [{name, default}] (default: string or undefined),
 * spanAttrs / resourceAttrs: Map, exclude: Set of the four fixed names.
 */
function buildKey(service, spanName, kind, status, dims = [], spanAttrs = new Map(),
  resourceAttrs = new Map(), exclude = new Set()) {
  return Buffer.from(buildKeyString(service, spanName, kind, status, dims, spanAttrs,
    resourceAttrs, exclude), 'utf8');
}

/** buildKey as a JS string (the connector's per-resource cache key). */
function buildKeyString(service, spanName, kind, status, dims = [], spanAttrs = new Map(),
  resourceAttrs = new Map(), exclude = new Set(), scope = null) {
  const parts = [];
  if (!exclude.has(SERVICE_NAME_KEY)) parts.push(service);
  if (!exclude.has(SPAN_NAME_KEY)) parts.push(spanName);
  if (!exclude.has(SPAN_KIND_KEY)) parts.push(spanKindStr(kind));
  if (!exclude.has(STATUS_CODE_KEY)) parts.push(statusCodeStr(status));
  let out = parts.join('\0');
  for (const d of dims) {
    let v;
    if (spanAttrs.has(d.name)) v = spanAttrs.get(d.name);
    else if (resourceAttrs.has(d.name)) v = resourceAttrs.get(d.name);
    else if (d.default !== undefined && d.default !== null) v = { type: 'string', value: String(d.default) };
    else continue;  // A5: a missing optional dimension is skipped with no separator
    out += '\0' + asString(v);
  }
  // include_instrumentation_scope: the span's scope name and version follow
  // the dimensions, both always present (an empty version keeps its separator)
  if (scope) out += '\0' + scope.name + '\0' + scope.version;
  return out;
}

const SCOPE_NAME_KEY = 'span.instrumentation.scope.name';
const SCOPE_VERSION_KEY = 'span.instrumentation.scope.version';

/**
 * The scope a span is keyed with under include_instrumentation_scope (a list
 * of scope names): {name, version} when the span's scope name is listed, else
 * null.  [UPSTREAM] connector.go buildKey / buildAttributes (confidence L:
 * not in /root/reference; no file there pins the option or its names).
 */
function includedScope(scope, names) {
  if (!names || names.size === 0 || !scope) return null;
  const name = scope.name || '';
  return names.has(name) ? { name, version: scope.version || '' } : null;
}

/** buildAttributes: datapoint attributes with dims copied with their original type (a7). */
function buildAttributes(service, spanName, kind, status, dims = [], spanAttrs = new Map(),
  resourceAttrs = new Map(), exclude = new Set(), scope = null) {
  const out = [];
  const str = (value) => ({ type: 'string', value });
  if (!exclude.has(SERVICE_NAME_KEY)) out.push({ key: SERVICE_NAME_KEY, value: str(service) });
  if (!exclude.has(SPAN_NAME_KEY)) out.push({ key: SPAN_NAME_KEY, value: str(spanName) });
  if (!exclude.has(SPAN_KIND_KEY)) out.push({ key: SPAN_KIND_KEY, value: str(spanKindStr(kind)) });
  if (!exclude.has(STATUS_CODE_KEY)) out.push({ key: STATUS_CODE_KEY, value: str(statusCodeStr(status)) });
  for (const d of dims) {
    if (spanAttrs.has(d.name)) out.push({ key: d.name, value: spanAttrs.get(d.name) });
    else if (resourceAttrs.has(d.name)) out.push({ key: d.name, value: resourceAttrs.get(d.name) });
    else if (d.default !== undefined && d.default !== null) out.push({ key: d.name, value: str(String(d.default)) });
  }
  if (scope) {
    out.push({ key: SCOPE_NAME_KEY, value: str(scope.name) });
    out.push({ key: SCOPE_VERSION_KEY, value: str(scope.version) });
  }
  return out;
}

/** Resource identity (stand-in for pdatautil.MapHash, = keys.py resource_hash). */
function resourceHash(resourceAttrs) {
  const keys = [...resourceAttrs.keys()].sort((a, b) => (Buffer.compare(Buffer.from(a), Buffer.from(b))));
  const chunks = [];
  for (const k of keys) {
    const v = resourceAttrs.get(k);
    chunks.push(Buffer.from(k, 'utf8'), Buffer.from([0]), Buffer.from(asString(v), 'utf8'),
      Buffer.from([0]), Buffer.from(TYPE_TAG[v.type] || 'NoneType', 'utf8'), Buffer.from([1]));
  }
  return xxh64(Buffer.concat(chunks), 0n);
}

/** xxh64(resource hash LE || key) with one seed. */
function seriesHashSeeded(resHash, key, seed) {
  const b = Buffer.alloc(8 + key.length);
  b.writeBigUInt64LE(resHash, 0);
  key.copy(b, 8);
  return xxh64(b, seed);
}

/**
 * Device series id of (resource, key): xxh64 with seed 0, 1, 2, ... until the
 * id is neither 0 (reserved by the engine) nor held by another series (a
 * 64-bit collision is re-salted, never shared).  owner(id) -> undefined
 * (free), true (this series already) or false (another series).  Returns
 * [id, seed].  Looks the hash up through module.exports so tests can force
 * collisions.
 */
function assignSeriesId(resHash, key, owner) {
  for (let seed = 0n; ; seed += 1n) {
    const h = module.exports.seriesHashSeeded(resHash, key, seed);
    if (h === 0n) continue;
    if (owner(h) !== false) return [h, seed];
  }
}

/** The id of a series with nothing else interned: seed 0 (seed 1 if that is 0). */
function seriesHash(resHash, key) {
  return assignSeriesId(resHash, key, () => undefined)[0];
}

/**
 * Series id -> {resHash, key, resourceAttrs, dpAttrs}; the first span seen
 * for an id fixes its datapoint attributes (A5/A6).  A distinct (resource,
 * key) whose id is taken is re-salted (counted in `collisions`).
 */
class KeyDictionary {
  constructor() { this.byId = new Map(); this.byKey = new Map(); this.collisions = 0; }
  intern(resHash, key, resourceAttrs, dpAttrs) {
    const name = `${resHash}:${key.toString('latin1')}`;
    const known = this.byKey.get(name);
    if (known !== undefined) return known;
    const [sid, seed] = assignSeriesId(resHash, key, (h) => {
      const cur = this.byId.get(h);
      return cur === undefined ? undefined : cur.resHash === resHash && Buffer.compare(cur.key, key) === 0;
    });
    if (seed > 0n) this.collisions += 1;
    if (!this.byId.has(sid)) this.byId.set(sid, { resHash, key, resourceAttrs, dpAttrs });
    this.byKey.set(name, sid);
    return sid;
  }
  get(sid) { return this.byId.get(sid); }
  get size() { return this.byId.size; }
}

module.exports = { SPAN_KIND_STR, STATUS_CODE_STR, SERVICE_NAME_KEY, spanKindStr, statusCodeStr,
  formatFloat, asString, attrMap, buildKey, buildKeyString, buildAttributes, includedScope,
  SCOPE_NAME_KEY, SCOPE_VERSION_KEY, resourceHash, seriesHash,
  seriesHashSeeded, assignSeriesId, KeyDictionary, useNativeXxh64 };
