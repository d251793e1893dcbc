'use strict';
/**
 * Minimal OTLP/protobuf codec for the host side of the connector (SURVEY.md
 * rows f1/f2): ExportTraceServiceRequest decode/encode (what the collector's
 * OTLP receiver hands the traces pipeline, /root/reference/src/otel-collector/
 * otelcol-config.yml:4-17) and ExportMetricsServiceRequest encode (what the
 * connector emits into the metrics pipeline, :118-127).
 *
 * Field numbers follow opentelemetry-proto v1 (trace/v1/trace.proto,
 * metrics/v1/metrics.proto, common/v1/common.proto, resource/v1/resource.proto).
 * Unknown fields are skipped on decode (proto3 forward compatibility).
 *
 * Decoded AnyValue = {type, value}, type in 'string' | 'bool' | 'int'
 * (BigInt) | 'double' | 'bytes' (Uint8Array) | 'array' (AnyValue[]) |
 * 'kvlist' ({key, value}[]) | 'empty' -- the shape keys.js consumes.
 */

const WT_VARINT = 0, WT_I64 = 1, WT_LEN = 2, WT_I32 = 5;
const utf8 = new TextDecoder('utf-8');

class Reader {
  constructor(buf, pos = 0, end = buf.length) {
    this.buf = buf; this.pos = pos; this.end = end;
  }
  eof() { return this.pos >= this.end; }
  byte() {
    if (this.pos >= this.end) throw new Error('protobuf: truncated message');
    return this.buf[this.pos++];
  }
  /** varint as a Number (exact below 2^53; used for tags, lengths, enums). */
  varint() {
    let x = 0, mul = 1;
    for (let i = 0; i < 10; i++) {
      const b = this.byte();
      x += (b & 0x7f) * mul;
      if (b < 0x80) return x;
      mul *= 128;
    }
    throw new Error('protobuf: varint too long');
  }
  /** varint as an unsigned 64-bit BigInt. */
  varint64() {
    let x = 0n, shift = 0n;
    for (let i = 0; i < 10; i++) {
      const b = this.byte();
      x |= BigInt(b & 0x7f) << shift;
      if (b < 0x80) return BigInt.asUintN(64, x);
      shift += 7n;
    }
    throw new Error('protobuf: varint too long');
  }
  need(n) {
    if (this.pos + n > this.end) throw new Error('protobuf: truncated message');
  }
  fixed64() {
    this.need(8);
    const v = this.buf.readBigUInt64LE(this.pos);
    this.pos += 8;
    return v;
  }
  fixed32() {
    this.need(4);
    const v = this.buf.readUInt32LE(this.pos);
    this.pos += 4;
    return v;
  }
  double() {
    this.need(8);
    const v = this.buf.readDoubleLE(this.pos);
    this.pos += 8;
    return v;
  }
  bytes() {
    const n = this.varint();
    this.need(n);
    const b = this.buf.subarray(this.pos, this.pos + n);
    this.pos += n;
    return b;
  }
  string() { return utf8.decode(this.bytes()); }
  sub() {
    const n = this.varint();
    this.need(n);
    const r = new Reader(this.buf, this.pos, this.pos + n);
    this.pos += n;
    return r;
  }
  skip(wt) {
    switch (wt) {
      case WT_VARINT: this.varint64(); break;
      case WT_I64: this.need(8); this.pos += 8; break;
      case WT_LEN: { const n = this.varint(); this.need(n); this.pos += n; break; }
      case WT_I32: this.need(4); this.pos += 4; break;
      default: throw new Error(`protobuf: unsupported wire type ${wt}`);
    }
  }
  /** Iterate fields: cb(fieldNumber, wireType) must consume or return false to skip. */
  fields(cb) {
    while (this.pos < this.end) {
      const tag = this.varint();
      const f = Math.floor(tag / 8), wt = tag & 7;
      if (f === 0) throw new Error('protobuf: field number 0');
      if (cb(f, wt) === false) this.skip(wt);
    }
  }
}

/** Nesting limit for array / kvlist values (as the native columnizer's kMaxAnyDepth). */
const MAX_ANY_DEPTH = 100;

function decodeArray(r, depth) {
  const out = [];
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { out.push(decodeAnyValue(r.sub(), depth + 1)); return true; }
    return false;
  });
  return out;
}

function decodeKvList(r, depth) {
  const out = [];
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { out.push(decodeKeyValue(r.sub(), depth + 1)); return true; }
    return false;
  });
  return out;
}

function decodeAnyValue(r, depth = 0) {
  if (depth > MAX_ANY_DEPTH) throw new Error('protobuf: attribute value nested too deeply');
  let v = { type: 'empty', value: null };
  r.fields((f, wt) => {
    switch (f) {
      case 1: if (wt !== WT_LEN) return false; v = { type: 'string', value: r.string() }; return true;
      case 2: if (wt !== WT_VARINT) return false; v = { type: 'bool', value: r.varint64() !== 0n }; return true;
      case 3: if (wt !== WT_VARINT) return false; v = { type: 'int', value: BigInt.asIntN(64, r.varint64()) }; return true;
      case 4: if (wt !== WT_I64) return false; v = { type: 'double', value: r.double() }; return true;
      case 5: if (wt !== WT_LEN) return false; v = { type: 'array', value: decodeArray(r.sub(), depth) }; return true;
      case 6: if (wt !== WT_LEN) return false; v = { type: 'kvlist', value: decodeKvList(r.sub(), depth) }; return true;
      case 7: if (wt !== WT_LEN) return false; v = { type: 'bytes', value: Uint8Array.from(r.bytes()) }; return true;
      default: return false;
    }
  });
  return v;
}

function decodeKeyValue(r, depth = 0) {
  let key = '', value = { type: 'empty', value: null };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { key = r.string(); return true; }
    if (f === 2 && wt === WT_LEN) { value = decodeAnyValue(r.sub(), depth); return true; }
    return false;
  });
  return { key, value };
}

function decodeStatus(r) {
  const s = { message: '', code: 0 };
  r.fields((f, wt) => {
    if (f === 2 && wt === WT_LEN) { s.message = r.string(); return true; }
    if (f === 3 && wt === WT_VARINT) { s.code = Number(BigInt.asIntN(32, r.varint64())); return true; }
    return false;
  });
  return s;
}

function decodeEvent(r) {
  const e = { timeUnixNano: 0n, name: '', attributes: [] };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_I64) { e.timeUnixNano = r.fixed64(); return true; }
    if (f === 2 && wt === WT_LEN) { e.name = r.string(); return true; }
    if (f === 3 && wt === WT_LEN) { e.attributes.push(decodeKeyValue(r.sub())); return true; }
    return false;
  });
  return e;
}

function decodeSpan(r) {
  const s = {
    traceId: new Uint8Array(16), spanId: new Uint8Array(8), parentSpanId: new Uint8Array(0),
    traceState: '', name: '', kind: 0, startTimeUnixNano: 0n, endTimeUnixNano: 0n,
    attributes: [], events: [], status: { message: '', code: 0 }, flags: 0,
  };
  r.fields((f, wt) => {
    switch (f) {
      case 1: if (wt !== WT_LEN) return false; s.traceId = Uint8Array.from(r.bytes()); return true;
      case 2: if (wt !== WT_LEN) return false; s.spanId = Uint8Array.from(r.bytes()); return true;
      case 3: if (wt !== WT_LEN) return false; s.traceState = r.string(); return true;
      case 4: if (wt !== WT_LEN) return false; s.parentSpanId = Uint8Array.from(r.bytes()); return true;
      case 5: if (wt !== WT_LEN) return false; s.name = r.string(); return true;
      case 6: if (wt !== WT_VARINT) return false; s.kind = Number(BigInt.asIntN(32, r.varint64())); return true;
      case 7: if (wt !== WT_I64) return false; s.startTimeUnixNano = r.fixed64(); return true;
      case 8: if (wt !== WT_I64) return false; s.endTimeUnixNano = r.fixed64(); return true;
      case 9: if (wt !== WT_LEN) return false; s.attributes.push(decodeKeyValue(r.sub())); return true;
      case 11: if (wt !== WT_LEN) return false; s.events.push(decodeEvent(r.sub())); return true;
      case 15: if (wt !== WT_LEN) return false; s.status = decodeStatus(r.sub()); return true;
      case 16: if (wt !== WT_I32) return false; s.flags = r.fixed32(); return true;
      default: return false;  // links, dropped counts: not used by the connector
    }
  });
  return s;
}

/** The fields of a Span an exemplar keeps (trace id, span id, start and end
 * times); every other field is skipped undecoded. */
function decodeSpanExemplar(r) {
  const s = { traceId: new Uint8Array(16), spanId: new Uint8Array(8), startTimeUnixNano: 0n, endTimeUnixNano: 0n };
  r.fields((f, wt) => {
    switch (f) {
      case 1: if (wt !== WT_LEN) return false; s.traceId = Uint8Array.from(r.bytes()); return true;
      case 2: if (wt !== WT_LEN) return false; s.spanId = Uint8Array.from(r.bytes()); return true;
      case 7: if (wt !== WT_I64) return false; s.startTimeUnixNano = r.fixed64(); return true;
      case 8: if (wt !== WT_I64) return false; s.endTimeUnixNano = r.fixed64(); return true;
      default: return false;
    }
  });
  return s;
}

function decodeResource(r) {
  const res = { attributes: [] };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { res.attributes.push(decodeKeyValue(r.sub())); return true; }
    return false;
  });
  return res;
}

function decodeScope(r) {
  const sc = { name: '', version: '', attributes: [] };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { sc.name = r.string(); return true; }
    if (f === 2 && wt === WT_LEN) { sc.version = r.string(); return true; }
    if (f === 3 && wt === WT_LEN) { sc.attributes.push(decodeKeyValue(r.sub())); return true; }
    return false;
  });
  return sc;
}

function decodeScopeSpans(r) {
  const ss = { scope: { name: '', version: '', attributes: [] }, spans: [], schemaUrl: '' };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { ss.scope = decodeScope(r.sub()); return true; }
    if (f === 2 && wt === WT_LEN) { ss.spans.push(decodeSpan(r.sub())); return true; }
    if (f === 3 && wt === WT_LEN) { ss.schemaUrl = r.string(); return true; }
    return false;
  });
  return ss;
}

function decodeResourceSpans(r) {
  const rs = { resource: { attributes: [] }, scopeSpans: [], schemaUrl: '' };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { rs.resource = decodeResource(r.sub()); return true; }
    if (f === 2 && wt === WT_LEN) { rs.scopeSpans.push(decodeScopeSpans(r.sub())); return true; }
    if (f === 3 && wt === WT_LEN) { rs.schemaUrl = r.string(); return true; }
    return false;
  });
  return rs;
}

/** ExportTraceServiceRequest bytes -> {resourceSpans: [...]}. */
function decodeTraces(buf) {
  const b = Buffer.isBuffer(buf) ? buf : Buffer.from(buf.buffer, buf.byteOffset, buf.byteLength);
  const r = new Reader(b);
  const req = { resourceSpans: [] };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { req.resourceSpans.push(decodeResourceSpans(r.sub())); return true; }
    return false;
  });
  return req;
}

// ---------------------------------------------------------------- encoding

class Writer {
  constructor() { this.chunks = []; this.len = 0; }
  push(b) { this.chunks.push(b); this.len += b.length; return this; }
  /** Unsigned varint of a Number or BigInt; negative values as 64-bit two's complement. */
  varint(v) {
    let x = typeof v === 'bigint' ? BigInt.asUintN(64, v) : (v < 0 ? BigInt.asUintN(64, BigInt(v)) : null);
    if (x === null) {
      if (v < 0x80) return this.push(Buffer.from([v]));
      x = BigInt(v);
    }
    const out = [];
    while (x >= 0x80n) { out.push(Number(x & 0x7fn) | 0x80); x >>= 7n; }
    out.push(Number(x));
    return this.push(Buffer.from(out));
  }
  tag(f, wt) { return this.varint(f * 8 + wt); }
  fixed64(v) { const b = Buffer.alloc(8); b.writeBigUInt64LE(BigInt.asUintN(64, BigInt(v))); return this.push(b); }
  fixed32(v) { const b = Buffer.alloc(4); b.writeUInt32LE(v >>> 0); return this.push(b); }
  double(v) { const b = Buffer.alloc(8); b.writeDoubleLE(v); return this.push(b); }
  bytes(b) { this.varint(b.length); return this.push(Buffer.from(b.buffer, b.byteOffset, b.byteLength)); }
  string(s) { return this.bytes(Buffer.from(s, 'utf8')); }
  finish() { return Buffer.concat(this.chunks, this.len); }

  // proto3 field helpers: default values are omitted, as the Go marshaller does
  fString(f, s) { if (s) this.tag(f, WT_LEN).string(s); return this; }
  fBytes(f, b) { if (b && b.length) this.tag(f, WT_LEN).bytes(b); return this; }
  fVarint(f, v) { if (v) this.tag(f, WT_VARINT).varint(v); return this; }
  fBool(f, v) { if (v) this.tag(f, WT_VARINT).varint(1); return this; }
  fFixed64(f, v) { if (v) this.tag(f, WT_I64).fixed64(v); return this; }
  fFixed32(f, v) { if (v) this.tag(f, WT_I32).fixed32(v); return this; }
  fSint32(f, v) { if (v) this.tag(f, WT_VARINT).varint(((v << 1) ^ (v >> 31)) >>> 0); return this; }
  fMsg(f, encodeFn, obj) {
    const w = new Writer();
    encodeFn(w, obj);
    const b = w.finish();
    return this.tag(f, WT_LEN).bytes(b);
  }
}

function encodeAnyValue(w, v) {
  switch (v.type) {
    case 'string': w.tag(1, WT_LEN).string(v.value); break;
    case 'bool': w.tag(2, WT_VARINT).varint(v.value ? 1 : 0); break;
    case 'int': w.tag(3, WT_VARINT).varint(BigInt(v.value)); break;
    case 'double': w.tag(4, WT_I64).double(v.value); break;
    case 'array': w.fMsg(5, (ww, arr) => { for (const x of arr) ww.fMsg(1, encodeAnyValue, x); }, v.value); break;
    case 'kvlist': w.fMsg(6, (ww, kvs) => { for (const kv of kvs) ww.fMsg(1, encodeKeyValue, kv); }, v.value); break;
    case 'bytes': w.tag(7, WT_LEN).bytes(v.value); break;
    default: break;  // empty AnyValue
  }
}

function encodeKeyValue(w, kv) {
  w.fString(1, kv.key);
  w.fMsg(2, encodeAnyValue, kv.value);
}

function encodeResource(w, res) {
  for (const kv of res.attributes || []) w.fMsg(1, encodeKeyValue, kv);
}

function encodeScope(w, sc) {
  w.fString(1, sc.name);
  w.fString(2, sc.version);
  for (const kv of sc.attributes || []) w.fMsg(3, encodeKeyValue, kv);
}

function encodeSpan(w, s) {
  w.fBytes(1, s.traceId);
  w.fBytes(2, s.spanId);
  w.fString(3, s.traceState);
  w.fBytes(4, s.parentSpanId);
  w.fString(5, s.name);
  w.fVarint(6, s.kind);
  w.fFixed64(7, s.startTimeUnixNano);
  w.fFixed64(8, s.endTimeUnixNano);
  for (const kv of s.attributes || []) w.fMsg(9, encodeKeyValue, kv);
  for (const ev of s.events || []) {
    w.fMsg(11, (ww, e) => {
      ww.fFixed64(1, e.timeUnixNano);
      ww.fString(2, e.name);
      for (const kv of e.attributes || []) ww.fMsg(3, encodeKeyValue, kv);
    }, ev);
  }
  const st = s.status || {};
  if (st.message || st.code) {
    w.fMsg(15, (ww, x) => { ww.fString(2, x.message); ww.fVarint(3, x.code); }, st);
  }
  w.fFixed32(16, s.flags);
}

/** {resourceSpans: [...]} -> ExportTraceServiceRequest bytes. */
function encodeTraces(req) {
  const w = new Writer();
  for (const rs of req.resourceSpans || []) {
    w.fMsg(1, (w1, x) => {
      w1.fMsg(1, encodeResource, x.resource || { attributes: [] });
      for (const ss of x.scopeSpans || []) {
        w1.fMsg(2, (w2, y) => {
          w2.fMsg(1, encodeScope, y.scope || {});
          for (const sp of y.spans || []) w2.fMsg(2, encodeSpan, sp);
          w2.fString(3, y.schemaUrl);
        }, ss);
      }
      w1.fString(3, x.schemaUrl);
    }, rs);
  }
  return w.finish();
}

const AGGREGATION_TEMPORALITY = { UNSPECIFIED: 0, DELTA: 1, CUMULATIVE: 2 };

function encodeNumberDataPoint(w, dp) {
  for (const kv of dp.attributes || []) w.fMsg(7, encodeKeyValue, kv);
  w.fFixed64(2, dp.startTimeUnixNano);
  w.fFixed64(3, dp.timeUnixNano);
  if (dp.asDouble !== undefined) w.tag(4, WT_I64).double(dp.asDouble);
  else w.tag(6, WT_I64).fixed64(BigInt.asUintN(64, BigInt(dp.asInt || 0n)));  // sfixed64
}

function encodeHistogramDataPoint(w, dp) {
  for (const kv of dp.attributes || []) w.fMsg(9, encodeKeyValue, kv);
  w.fFixed64(2, dp.startTimeUnixNano);
  w.fFixed64(3, dp.timeUnixNano);
  w.fFixed64(4, dp.count);
  if (dp.sum !== undefined) w.tag(5, WT_I64).double(dp.sum);  // optional: presence kept
  if (dp.bucketCounts && dp.bucketCounts.length) {
    const b = Buffer.alloc(8 * dp.bucketCounts.length);
    dp.bucketCounts.forEach((c, i) => b.writeBigUInt64LE(BigInt.asUintN(64, BigInt(c)), 8 * i));
    w.tag(6, WT_LEN).bytes(b);
  }
  if (dp.explicitBounds && dp.explicitBounds.length) {
    const b = Buffer.alloc(8 * dp.explicitBounds.length);
    dp.explicitBounds.forEach((x, i) => b.writeDoubleLE(x, 8 * i));
    w.tag(7, WT_LEN).bytes(b);
  }
  for (const ex of dp.exemplars || []) w.fMsg(8, encodeExemplar, ex);
}

function encodeExpoBuckets(w, b) {
  w.fSint32(1, b.offset || 0);
  const counts = b.bucketCounts || [];
  if (counts.length) {
    const p = new Writer();
    for (const c of counts) p.varint(BigInt(c));
    w.tag(2, WT_LEN).bytes(p.finish());
  }
}

/** ExponentialHistogramDataPoint (metrics.proto v1); positive/negative always
 * present, as pdata's non-nullable Buckets marshal. */
function encodeExpoHistogramDataPoint(w, dp) {
  for (const kv of dp.attributes || []) w.fMsg(1, encodeKeyValue, kv);
  w.fFixed64(2, dp.startTimeUnixNano);
  w.fFixed64(3, dp.timeUnixNano);
  w.fFixed64(4, dp.count);
  if (dp.sum !== undefined) w.tag(5, WT_I64).double(dp.sum);
  w.fSint32(6, dp.scale || 0);
  w.fFixed64(7, dp.zeroCount);
  w.fMsg(8, encodeExpoBuckets, dp.positive || {});
  w.fMsg(9, encodeExpoBuckets, dp.negative || {});
  for (const ex of dp.exemplars || []) w.fMsg(11, encodeExemplar, ex);
  if (dp.min !== undefined) w.tag(12, WT_I64).double(dp.min);
  if (dp.max !== undefined) w.tag(13, WT_I64).double(dp.max);
}

function encodeExemplar(w, ex) {
  w.fFixed64(2, ex.timeUnixNano);
  if (ex.asInt !== undefined) w.tag(6, WT_I64).fixed64(BigInt.asUintN(64, BigInt(ex.asInt)));
  else w.tag(3, WT_I64).double(ex.asDouble || 0);
  w.fBytes(4, ex.spanId);
  w.fBytes(5, ex.traceId);
  for (const kv of ex.filteredAttributes || []) w.fMsg(7, encodeKeyValue, kv);
}

function encodeMetric(w, m) {
  w.fString(1, m.name);
  w.fString(2, m.description);
  w.fString(3, m.unit);
  if (m.gauge) {
    w.fMsg(5, (ww, g) => {
      for (const dp of g.dataPoints || []) ww.fMsg(1, encodeNumberDataPoint, dp);
    }, m.gauge);
  } else if (m.sum) {
    w.fMsg(7, (ww, s) => {
      for (const dp of s.dataPoints || []) ww.fMsg(1, encodeNumberDataPoint, dp);
      ww.fVarint(2, s.aggregationTemporality);
      ww.fBool(3, s.isMonotonic);
    }, m.sum);
  } else if (m.histogram) {
    w.fMsg(9, (ww, h) => {
      for (const dp of h.dataPoints || []) ww.fMsg(1, encodeHistogramDataPoint, dp);
      ww.fVarint(2, h.aggregationTemporality);
    }, m.histogram);
  } else if (m.exponentialHistogram) {
    w.fMsg(10, (ww, h) => {
      for (const dp of h.dataPoints || []) ww.fMsg(1, encodeExpoHistogramDataPoint, dp);
      ww.fVarint(2, h.aggregationTemporality);
    }, m.exponentialHistogram);
  }
}

/** {resourceMetrics: [{resource, scopeMetrics: [{scope, metrics}]}]} -> ExportMetricsServiceRequest bytes. */
function encodeMetrics(req) {
  const w = new Writer();
  for (const rm of req.resourceMetrics || []) {
    w.fMsg(1, (w1, x) => {
      w1.fMsg(1, encodeResource, x.resource || { attributes: [] });
      for (const sm of x.scopeMetrics || []) {
        w1.fMsg(2, (w2, y) => {
          w2.fMsg(1, encodeScope, y.scope || {});
          for (const m of y.metrics || []) w2.fMsg(2, encodeMetric, m);
          w2.fString(3, y.schemaUrl);
        }, sm);
      }
      w1.fString(3, x.schemaUrl);
    }, rm);
  }
  return w.finish();
}

// --------------------------------------------------- metrics decode (tests)

function decodeNumberDataPoint(r) {
  const dp = { attributes: [], startTimeUnixNano: 0n, timeUnixNano: 0n };
  r.fields((f, wt) => {
    if (f === 7 && wt === WT_LEN) { dp.attributes.push(decodeKeyValue(r.sub())); return true; }
    if (f === 2 && wt === WT_I64) { dp.startTimeUnixNano = r.fixed64(); return true; }
    if (f === 3 && wt === WT_I64) { dp.timeUnixNano = r.fixed64(); return true; }
    if (f === 4 && wt === WT_I64) { dp.asDouble = r.double(); return true; }
    if (f === 6 && wt === WT_I64) { dp.asInt = BigInt.asIntN(64, r.fixed64()); return true; }
    return false;
  });
  return dp;
}

function decodePackedFixed64(r, wt, out, asDouble) {
  if (wt === WT_LEN) {
    const s = r.sub();
    while (!s.eof()) out.push(asDouble ? s.double() : s.fixed64());
  } else if (wt === WT_I64) {
    out.push(asDouble ? r.double() : r.fixed64());
  } else {
    return false;
  }
  return true;
}

function decodeExemplar(r) {
  const ex = { timeUnixNano: 0n, spanId: new Uint8Array(0), traceId: new Uint8Array(0), filteredAttributes: [] };
  r.fields((f, wt) => {
    if (f === 2 && wt === WT_I64) { ex.timeUnixNano = r.fixed64(); return true; }
    if (f === 3 && wt === WT_I64) { ex.asDouble = r.double(); return true; }
    if (f === 6 && wt === WT_I64) { ex.asInt = BigInt.asIntN(64, r.fixed64()); return true; }
    if (f === 4 && wt === WT_LEN) { ex.spanId = Uint8Array.from(r.bytes()); return true; }
    if (f === 5 && wt === WT_LEN) { ex.traceId = Uint8Array.from(r.bytes()); return true; }
    if (f === 7 && wt === WT_LEN) { ex.filteredAttributes.push(decodeKeyValue(r.sub())); return true; }
    return false;
  });
  return ex;
}

function decodeHistogramDataPoint(r) {
  const dp = { attributes: [], startTimeUnixNano: 0n, timeUnixNano: 0n, count: 0n,
    bucketCounts: [], explicitBounds: [] };
  r.fields((f, wt) => {
    if (f === 9 && wt === WT_LEN) { dp.attributes.push(decodeKeyValue(r.sub())); return true; }
    if (f === 2 && wt === WT_I64) { dp.startTimeUnixNano = r.fixed64(); return true; }
    if (f === 3 && wt === WT_I64) { dp.timeUnixNano = r.fixed64(); return true; }
    if (f === 4 && wt === WT_I64) { dp.count = r.fixed64(); return true; }
    if (f === 5 && wt === WT_I64) { dp.sum = r.double(); return true; }
    if (f === 8 && wt === WT_LEN) { (dp.exemplars = dp.exemplars || []).push(decodeExemplar(r.sub())); return true; }
    if (f === 6) return decodePackedFixed64(r, wt, dp.bucketCounts, false);
    if (f === 7) return decodePackedFixed64(r, wt, dp.explicitBounds, true);
    return false;
  });
  return dp;
}

function decodeExpoBuckets(r) {
  const b = { offset: 0, bucketCounts: [] };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_VARINT) { const z = r.varint(); b.offset = z % 2 ? -(z + 1) / 2 : z / 2; return true; }
    if (f === 2 && wt === WT_LEN) { const s = r.sub(); while (!s.eof()) b.bucketCounts.push(s.varint64()); return true; }
    if (f === 2 && wt === WT_VARINT) { b.bucketCounts.push(r.varint64()); return true; }
    return false;
  });
  return b;
}

function decodeExpoHistogramDataPoint(r) {
  const dp = { attributes: [], startTimeUnixNano: 0n, timeUnixNano: 0n, count: 0n, scale: 0, zeroCount: 0n,
    positive: { offset: 0, bucketCounts: [] }, negative: { offset: 0, bucketCounts: [] } };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { dp.attributes.push(decodeKeyValue(r.sub())); return true; }
    if (f === 2 && wt === WT_I64) { dp.startTimeUnixNano = r.fixed64(); return true; }
    if (f === 3 && wt === WT_I64) { dp.timeUnixNano = r.fixed64(); return true; }
    if (f === 4 && wt === WT_I64) { dp.count = r.fixed64(); return true; }
    if (f === 5 && wt === WT_I64) { dp.sum = r.double(); return true; }
    if (f === 6 && wt === WT_VARINT) { const z = r.varint(); dp.scale = z % 2 ? -(z + 1) / 2 : z / 2; return true; }
    if (f === 7 && wt === WT_I64) { dp.zeroCount = r.fixed64(); return true; }
    if (f === 8 && wt === WT_LEN) { dp.positive = decodeExpoBuckets(r.sub()); return true; }
    if (f === 9 && wt === WT_LEN) { dp.negative = decodeExpoBuckets(r.sub()); return true; }
    if (f === 11 && wt === WT_LEN) { (dp.exemplars = dp.exemplars || []).push(decodeExemplar(r.sub())); return true; }
    if (f === 12 && wt === WT_I64) { dp.min = r.double(); return true; }
    if (f === 13 && wt === WT_I64) { dp.max = r.double(); return true; }
    return false;
  });
  return dp;
}

function decodeMetric(r) {
  const m = { name: '', description: '', unit: '' };
  r.fields((f, wt) => {
    if (f === 1 && wt === WT_LEN) { m.name = r.string(); return true; }
    if (f === 2 && wt === WT_LEN) { m.description = r.string(); return true; }
    if (f === 3 && wt === WT_LEN) { m.unit = r.string(); return true; }
    if (f === 10 && wt === WT_LEN) {
      const body = { dataPoints: [], aggregationTemporality: 0 };
      const s = r.sub();
      s.fields((g, wt2) => {
        if (g === 1 && wt2 === WT_LEN) { body.dataPoints.push(decodeExpoHistogramDataPoint(s.sub())); return true; }
        if (g === 2 && wt2 === WT_VARINT) { body.aggregationTemporality = s.varint(); return true; }
        return false;
      });
      m.exponentialHistogram = body;
      return true;
    }
    if ((f === 5 || f === 7 || f === 9) && wt === WT_LEN) {
      const body = { dataPoints: [] };
      if (f !== 5) body.aggregationTemporality = 0;
      const s = r.sub();
      s.fields((g, wt2) => {
        if (g === 1 && wt2 === WT_LEN) {
          body.dataPoints.push(f === 9 ? decodeHistogramDataPoint(s.sub()) : decodeNumberDataPoint(s.sub()));
          return true;
        }
        if (g === 2 && wt2 === WT_VARINT && f !== 5) { body.aggregationTemporality = s.varint(); return true; }
        if (g === 3 && wt2 === WT_VARINT && f === 7) { body.isMonotonic = s.varint() !== 0; return true; }
        return false;
      });
      if (f === 5) m.gauge = body;
      else if (f === 7) { body.isMonotonic = !!body.isMonotonic; m.sum = body; } else m.histogram = body;
      return true;
    }
    return false;
  });
  return m;
}

/** ExportMetricsServiceRequest bytes -> {resourceMetrics: [...]} (Gauge, Sum, Histogram, ExponentialHistogram). */
function decodeMetrics(buf) {
  const b = Buffer.isBuffer(buf) ? buf : Buffer.from(buf.buffer, buf.byteOffset, buf.byteLength);
  const r = new Reader(b);
  const req = { resourceMetrics: [] };
  r.fields((f, wt) => {
    if (f !== 1 || wt !== WT_LEN) return false;
    const rm = { resource: { attributes: [] }, scopeMetrics: [], schemaUrl: '' };
    const x = r.sub();
    x.fields((g, wt2) => {
      if (g === 1 && wt2 === WT_LEN) { rm.resource = decodeResource(x.sub()); return true; }
      if (g === 3 && wt2 === WT_LEN) { rm.schemaUrl = x.string(); return true; }
      if (g !== 2 || wt2 !== WT_LEN) return false;
      const sm = { scope: { name: '', version: '', attributes: [] }, metrics: [], schemaUrl: '' };
      const y = x.sub();
      y.fields((h, wt3) => {
        if (h === 1 && wt3 === WT_LEN) { sm.scope = decodeScope(y.sub()); return true; }
        if (h === 2 && wt3 === WT_LEN) { sm.metrics.push(decodeMetric(y.sub())); return true; }
        if (h === 3 && wt3 === WT_LEN) { sm.schemaUrl = y.string(); return true; }
        return false;
      });
      rm.scopeMetrics.push(sm);
      return true;
    });
    req.resourceMetrics.push(rm);
    return true;
  });
  return req;
}

module.exports = { Reader, Writer, decodeAnyValue, decodeKeyValue, decodeSpan, decodeSpanExemplar, decodeResource, decodeTraces,
  encodeAnyValue, encodeKeyValue, encodeSpan, encodeTraces, encodeMetrics, decodeMetrics,
  AGGREGATION_TEMPORALITY };
