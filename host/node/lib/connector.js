'use strict';
/**
 * SpanMetricsConnector -- the Node host of the spanmetrics connector, with the
 * per-span aggregation on the GPU through the N-API addon (SURVEY.md 8b).
 *
 * Mirrors the upstream component ([UPSTREAM] opentelemetry-collector-contrib
 * connector/spanmetricsconnector v0.125.0, wired by
 * /root/reference/src/otel-collector/otelcol-config.yml:115-127):
 *
 *   upstream (Go)                          here
 *   -------------------------------------  ---------------------------------------
 *   createDefaultConfig / Config           normalizeConfig (YAML field names)
 *   createTracesToMetricsConnector + Start constructor + start()
 *   ConsumeTraces -> aggregateMetrics      consumeTraces (keys on the host, the
 *                                          numeric work in addon.ingest)
 *   exportMetrics -> buildMetrics          exportMetrics (addon.flush delta ->
 *     + resetState                         cumulative/delta OTLP metrics)
 *   getOrCreateResourceMetrics + LRU       _resource (LRU with evicted side map)
 *   Shutdown                               shutdown()
 *   (new) HLL / count-min windows          windowSketch / sketch metrics
 *
 * The host owns the string world (keys, attributes, resources); the device sees
 * only u64 series ids (keys.js seriesHash) in SoA v1 columns.  Spans are
 * columnised into a reusable buffer and handed to the engine when it fills
 * (`batch_size` spans) or at export -- the batching the demo's `batch`
 * processor does upstream of the connector (otelcol-config.yml:100,121).
 */
const addonLoader = require('./addon');
const keys = require('./keys');
const otlp = require('./otlp');
const expohisto = require('./expohisto');
const { applyRules } = require('./transform');

const M64 = (1n << 64n) - 1n;
const CMS_SEED = [0x9E3779B97F4A7C15n, 0xBF58476D1CE4E5B9n, 0x94D049BB133111EBn,
  0xD6E8FEB86659FD93n, 0xA0761D6478BD642Fn, 0xE7037ED1A0B428DBn, 0x8EBC6AF09C88C6E3n,
  0x589965CC75374CC3n];

/** splitmix64 finaliser (the count-min column hash, SURVEY.md a17). */
function splitmix64(x) {
  let z = (x + 0x9E3779B97F4A7C15n) & M64;
  z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & M64;
  z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & M64;
  return z ^ (z >> 31n);
}

const DUR_UNITS = { ns: 1, us: 1e3, 'µs': 1e3, 'μs': 1e3, ms: 1e6, s: 1e9, m: 60e9, h: 3600e9 };

/** Go time.ParseDuration subset ("2ms", "1.5s", "1m30s") -> nanoseconds (Number). */
function parseDurationNs(s) {
  if (typeof s === 'number') return s;
  const str = String(s).trim();
  if (str === '0') return 0;
  const re = /(\d+(?:\.\d*)?|\.\d+)(ns|us|µs|μs|ms|s|m|h)/gy;
  let total = 0, m, pos = 0, sign = 1, body = str;
  if (body[0] === '-' || body[0] === '+') { sign = body[0] === '-' ? -1 : 1; body = body.slice(1); }
  re.lastIndex = 0;
  while (pos < body.length && (m = re.exec(body)) !== null) {
    total += parseFloat(m[1]) * DUR_UNITS[m[2]];
    pos = re.lastIndex;
  }
  if (pos !== body.length || pos === 0) throw new Error(`invalid duration ${JSON.stringify(s)}`);
  return sign * total;
}

// reserved key strings (a real key never starts with U+0001 / U+0002)
const OVERFLOW_KEY = '\u0001otel.metric.overflow';
const EVENT_KEY_PREFIX = '\u0002events\u0000';
// calls_dimensions / histogram.dimensions: the calls and the duration metric
// keep separate series (upstream: separate sums and histograms maps), keyed
// in their own namespaces
const CALLS_KEY_PREFIX = '\u0003calls\u0000';
// series kinds whose records feed the sketches (see _pushCalls, _pushEvent)
const SKETCH_KINDS = new Set(['span', 'overflow', 'hist', 'hist-overflow']);
const HIST_KEY_PREFIX = '\u0004hist\u0000';

const NONE = [];
const asBuffer = (b) => (Buffer.isBuffer(b) ? b : Buffer.from(b.buffer, b.byteOffset, b.byteLength));

const TEMPORALITY = {
  AGGREGATION_TEMPORALITY_CUMULATIVE: otlp.AGGREGATION_TEMPORALITY.CUMULATIVE,
  AGGREGATION_TEMPORALITY_DELTA: otlp.AGGREGATION_TEMPORALITY.DELTA,
};

/**
 * Config with the spanmetrics YAML field names; defaults = createDefaultConfig
 * (the reference declares `spanmetrics:` with an empty body, SURVEY.md a1).
 * `sketches`, `key_capacity`, `device`, `devices`, `batch_size` are this
 * build's own; `devices: [0, 1, ...]` runs one engine per listed GPU behind the
 * connector (spans sharded by trace id, merged at every flush and window read).
 * Histogram buckets: duration strings ("2ms") as in YAML, or numbers already
 * in the histogram unit.
 */
function normalizeConfig(cfg = {}, addon) {
  const d = addon.configDefault();
  const hist = cfg.histogram || {};
  const unit = hist.unit || 'ms';
  if (unit !== 'ms' && unit !== 's') throw new Error(`histogram.unit must be ms or s, got ${unit}`);
  if (hist.exponential && hist.explicit) throw new Error('use either `explicit` or `exponential` buckets histogram');
  // go-expohisto structure.DefaultMaxSize when max_size is unset; the engine takes 2..4096
  const expMaxSize = hist.exponential ? (hist.exponential.max_size || 160) : 0;
  if (hist.exponential && !(Number.isInteger(expMaxSize) && expMaxSize >= 2 && expMaxSize <= 4096)) {
    throw new Error(`histogram.exponential.max_size must be 2..4096, got ${hist.exponential.max_size}`);
  }
  const div = unit === 's' ? 1e9 : 1e6;
  let bounds = d.bounds.slice();
  if (hist.explicit && Array.isArray(hist.explicit.buckets)) {
    // durationsToUnits: float64(d.Nanoseconds()) / unitDivider
    bounds = hist.explicit.buckets.map((b) => (typeof b === 'number' ? b : parseDurationNs(b) / div));
  }
  const temporality = cfg.aggregation_temporality || 'AGGREGATION_TEMPORALITY_CUMULATIVE';
  if (!(temporality in TEMPORALITY)) throw new Error(`unknown aggregation_temporality ${temporality}`);
  const dimList = (l) => (l || []).map((x) => ({ name: x.name,
    default: x.default === undefined || x.default === null ? undefined : String(x.default) }));
  const dims = dimList(cfg.dimensions);
  // [UPSTREAM] config.go (confidence M): calls_dimensions and histogram.dimensions
  // add dimensions to one metric only, after `dimensions`
  const callsDims = dims.concat(dimList(cfg.calls_dimensions));
  const histDims = dims.concat(dimList(hist.dimensions));
  const sk = cfg.sketches || {};
  const windowNs = sk.window !== undefined ? BigInt(Math.round(parseDurationNs(sk.window))) : d.windowNs;
  return {
    unit, bounds, dims, expMaxSize, callsDims, histDims,
    splitKeys: callsDims.length !== dims.length || histDims.length !== dims.length,
    // include_instrumentation_scope: scope names whose spans are keyed with
    // their scope's name and version ([UPSTREAM] config.go, confidence L)
    scopes: new Set(cfg.include_instrumentation_scope || []),
    // histogram.disable: no duration metric (the calls metric stays)
    histogramDisable: !!hist.disable,
    // metrics_expiration: cumulative resources not seen for this long are
    // exported one last time and then dropped (0: never)
    expirationNs: cfg.metrics_expiration !== undefined ? BigInt(Math.round(parseDurationNs(cfg.metrics_expiration))) : 0n,
    exclude: new Set(cfg.exclude_dimensions || []),
    temporality: TEMPORALITY[temporality],
    namespace: cfg.namespace === undefined ? 'traces.span.metrics' : cfg.namespace,
    flushIntervalMs: cfg.metrics_flush_interval !== undefined
      ? parseDurationNs(cfg.metrics_flush_interval) / 1e6 : 60000,
    resourceCacheSize: cfg.resource_metrics_cache_size || 1000,
    resourceKeyAttributes: cfg.resource_metrics_key_attributes || [],
    hllP: sk.hll_p || d.hllP, cmsD: sk.cms_d || d.cmsD, cmsW: sk.cms_w || d.cmsW,
    windowNs, nWindows: sk.n_windows || d.nWindows, nServices: sk.n_services || d.nServices,
    emitSketches: !!sk.emit, topK: sk.top_k || 10,
    cardinalityLimit: cfg.aggregation_cardinality_limit || 0,
    exemplars: !!(cfg.exemplars && cfg.exemplars.enabled),
    exemplarsMax: (cfg.exemplars && cfg.exemplars.max_per_data_point) || 5,
    events: !!(cfg.events && cfg.events.enabled),
    eventDims: ((cfg.events && cfg.events.dimensions) || []).map((x) => ({ name: x.name,
      default: x.default === undefined || x.default === null ? undefined : String(x.default) })),
    keyCapacity: cfg.key_capacity || d.keyCapacity,
    device: cfg.device || 0,
    devices: Array.isArray(cfg.devices) && cfg.devices.length ? cfg.devices.map(Number) : null,
    batchSize: cfg.batch_size || 1 << 16,
    // native columnizer worker threads for consumeTracesBatch (this build's own)
    columnizerThreads: cfg.columnizer_threads !== undefined ? cfg.columnizer_threads
      : Math.min(8, require('os').cpus().length),
  };
}

/** Reusable SoA v1 column buffer (44 B/span). */
class Columns {
  constructor(cap) {
    this.cap = cap;
    this.n = 0;
    this.keyHash = new BigUint64Array(cap);
    this.startNs = new BigUint64Array(cap);
    this.endNs = new BigUint64Array(cap);
    this.traceW0 = new BigUint64Array(cap);
    this.traceW1 = new BigUint64Array(cap);
    this.meta = new Uint32Array(cap);
    this.w0u8 = new Uint8Array(this.traceW0.buffer);
    this.w1u8 = new Uint8Array(this.traceW1.buffer);
  }
  view() {
    const n = this.n;
    return { keyHash: this.keyHash.subarray(0, n), startNs: this.startNs.subarray(0, n),
      endNs: this.endNs.subarray(0, n), traceW0: this.traceW0.subarray(0, n),
      traceW1: this.traceW1.subarray(0, n), meta: this.meta.subarray(0, n) };
  }
}

class SpanMetricsConnector {
  /**
   * @param cfg spanmetrics YAML-shaped config (see normalizeConfig)
   * @param opts {addon, clock: () => BigInt ns, metricsConsumer: (req) => void,
   *              rules: span-name rules applied before keying (transform.js),
   *              native: false to force the JavaScript columnizer}
   */
  constructor(cfg = {}, opts = {}) {
    this.addon = opts.addon || addonLoader.load();
    this.cfg = normalizeConfig(cfg, this.addon);
    this.rules = opts.rules || [];
    this.clock = opts.clock || (() => BigInt(Date.now()) * 1000000n);
    this.metricsConsumer = opts.metricsConsumer || null;
    const c = this.cfg;
    this.handle = this.addon.create({ bounds: c.bounds, unit: c.unit, hllP: c.hllP, cmsD: c.cmsD,
      cmsW: c.cmsW, windowNs: c.windowNs, nWindows: c.nWindows, nServices: c.nServices,
      keyCapacity: c.keyCapacity, device: c.device, expMaxSize: c.expMaxSize, ...(c.devices ? { devices: c.devices } : {}) });
    this.cols = new Columns(c.batchSize);
    // native OTLP columnizer (binding/otlp_columnizer.cc) for request bytes
    // (dimensions, exclusions, rules, resource key attributes, the cardinality
    // limit, exemplars and events are all native); the JS path below takes the
    // requests it reports as fallbacks
    this.col = null;
    this.nativeMaxEnd = 0n;
    this.nativeBuffered = 0;
    this.nativeRequests = 0;
    this.jsRequests = 0;
    // (calls_dimensions / histogram.dimensions key every span twice, and
    // include_instrumentation_scope keys by the scope: the JavaScript
    // columnizer does both)
    if (opts.native !== false && typeof this.addon.createColumnizer === 'function' &&
        this.rules.every((r) => r.native) && !c.splitKeys && c.scopes.size === 0) {
      this.col = this.addon.createColumnizer(this.handle, { dims: c.dims,
        exclude: [...c.exclude], rules: this.rules.map((r) => r.native),
        keyAttributes: c.resourceKeyAttributes, threads: c.columnizerThreads,
        cardinalityLimit: c.cardinalityLimit, exemplars: c.exemplars, exemplarsMax: c.exemplarsMax,
        events: c.events, eventDims: c.eventDims });
    }
    this.resources = new Map();   // resHash -> resource record (LRU order: oldest first)
    this.evicted = new Map();     // evicted this flush interval, revivable until export
    this.series = new Map();      // sid -> series record
    this.services = new Map();    // service.name -> service id (first-seen order)
    this.lastDeltaTs = new Map(); // sid -> last delta export timestamp
    this.windowBase = null;
    this.maxWindowSeen = -1n;
    this.sketchWatermark = 0n;
    this.closedWindows = [];
    this.droppedFlushes = 0;
    this.droppedSpans = 0n;       // the engine's dropped_table_full after the last dropping flush
    this.onDrop = opts.onDrop || null;
    this.collisions = 0;          // series ids re-salted after a 64-bit collision
    this._verifyingNative = false;
    this.eventRecords = 0;
    this.callsRecords = 0;  // calls-series records of split keys (_pushCalls)
    this.nativeRemaps = 0;  // native series ids the host dictionary replaced (collisions)
    this.ticker = null;
  }

  capabilities() { return { mutatesData: false }; }

  /** Start: the flush ticker (metrics_flush_interval) feeding metricsConsumer. */
  start() {
    if (this.ticker || !this.metricsConsumer) return;
    this.ticker = setInterval(() => {
      // export failures are the consumer's to count; the ticker keeps going
      Promise.resolve().then(() => this.metricsConsumer(this.exportMetrics())).catch(() => {});
    }, this.cfg.flushIntervalMs);
    if (this.ticker.unref) this.ticker.unref();
  }

  shutdown() {
    if (this.ticker) clearInterval(this.ticker);
    this.ticker = null;
    if (this.col && this.addon.columnizerDestroy) this.addon.columnizerDestroy(this.col);
    this.col = null;
    if (this.handle) this.addon.destroy(this.handle);
    this.handle = null;
  }

  // ------------------------------------------------------------ ingest

  _serviceId(name) {
    let id = this.services.get(name);
    if (id === undefined) {
      // one numbering for both columnizers: the native one owns it when present
      id = this.col ? this.addon.columnizerServiceId(this.col, name)[0]
        : Math.min(this.services.size, 0xFFFE);  // 0xFFFF: event records (no sketch)
      this.services.set(name, id);
    }
    return id;
  }

  /** getOrCreateResourceMetrics: LRU(resource_metrics_cache_size) + evicted side map. */
  _resource(resAttrs) {
    const keyAttrs = this.cfg.resourceKeyAttributes;
    let hashAttrs = resAttrs;
    if (keyAttrs.length) {
      hashAttrs = new Map();
      for (const k of keyAttrs) if (resAttrs.has(k)) hashAttrs.set(k, resAttrs.get(k));
    }
    const h = keys.resourceHash(hashAttrs);
    return this._touchResource(h) ||
      this._admitResource({ hash: h, attributes: resAttrs, startTs: this.clock(), byKey: new Map(),
        sids: [], nSpanSeries: 0, nByKind: {} });
  }

  /**
   * The attributes of the resource a natively keyed span came from: its own
   * Resource message when dimensions are configured (resources that share a
   * resource hash -- resource_metrics_key_attributes -- can differ in the
   * attributes a dimension reads, as the JavaScript path keys them), else the
   * resource entry's.
   */
  _spanResourceAttrs(bytes, rec, res) {
    if (!this.cfg.dims.length || rec.resOff === undefined) return res.attributes;
    if (rec.resOff < 0) return new Map();
    return keys.attrMap(otlp.decodeResource(new otlp.Reader(bytes, rec.resOff, rec.resOff + rec.resLen)).attributes);
  }

  /** LRU hit (or revival from the evicted side map) by resource hash; undefined on a miss. */
  _touchResource(h) {
    let r = this.resources.get(h);
    if (r !== undefined) {
      this.resources.delete(h);  // refresh LRU position
      this.resources.set(h, r);
      if (this.cfg.expirationNs) r.lastSeen = this.clock();
      return r;
    }
    r = this.evicted.get(h);
    if (r === undefined) return undefined;
    this.evicted.delete(h);
    return this._admitResource(r);
  }

  _admitResource(r) {
    if (this.cfg.expirationNs) r.lastSeen = this.clock();
    this.resources.set(r.hash, r);
    if (this.resources.size > this.cfg.resourceCacheSize) {
      const [oldest, rec] = this.resources.entries().next().value;
      this.resources.delete(oldest);
      this.evicted.set(oldest, rec);  // the native side keeps its keys until export drops it
    }
    return r;
  }

  /**
   * Series id of a key string in a resource, interning it on first sight.
   * `mkAttrs` builds the datapoint attributes (called once per key: the first
   * span seen fixes them, A5/A6).  kind: 'span' | 'event' | 'overflow'.
   */
  _intern(res, keyStr, kind, status, mkAttrs) {
    let sid = res.byKey.get(keyStr);
    if (sid !== undefined) return sid;
    const keyBuf = Buffer.from(keyStr, 'utf8');
    // a 64-bit collision with another series is re-salted (ConsumeTraces never fails)
    let seed;
    [sid, seed] = keys.assignSeriesId(res.hash, keyBuf, (h) => {
      const s = this.series.get(h);
      return s === undefined ? undefined : s.res.hash === res.hash && s.keyStr === keyStr;
    });
    if (seed > 0n) this.collisions += 1;
    const cur = this.series.get(sid);
    // the native columnizer learns series the JavaScript path saw first
    if (cur === undefined && this.col && !this._verifyingNative) {
      this.addon.columnizerLearn(this.col, res.hash, keyBuf, sid);
    }
    if (cur === undefined) {
      this.series.set(sid, { sid, res, keyStr, dpAttrs: mkAttrs(), status, kind,
        counts: null, sumNs: 0n, exemplars: [] });
      res.sids.push(sid);
      if (kind === 'span') res.nSpanSeries += 1;
      res.nByKind[kind] = (res.nByKind[kind] || 0) + 1;
    }
    res.byKey.set(keyStr, sid);
    return sid;
  }

  _seriesId(res, service, span, resAttrs, spanAttrs, scope = null) {
    const c = this.cfg;
    const status = span.status ? span.status.code : 0;
    if (c.splitKeys) return this._splitId(res, service, span, resAttrs, spanAttrs, status, HIST_KEY_PREFIX, scope);
    const keyStr = keys.buildKeyString(service, span.name, span.kind, status, c.dims, spanAttrs,
      resAttrs, c.exclude, scope);
    const known = res.byKey.get(keyStr);
    if (known !== undefined) return known;
    // aggregation_cardinality_limit: past `limit` series in a resource, new keys
    // share one overflow series (attribute otel.metric.overflow = true)
    if (c.cardinalityLimit > 0 && res.nSpanSeries >= c.cardinalityLimit) {
      return this._intern(res, OVERFLOW_KEY, 'overflow', 0,
        () => [{ key: 'otel.metric.overflow', value: { type: 'bool', value: true } }]);
    }
    return this._intern(res, keyStr, 'span', status, () => keys.buildAttributes(service, span.name,
      span.kind, status, c.dims, spanAttrs, resAttrs, c.exclude, scope));
  }

  /**
   * calls_dimensions / histogram.dimensions: the span's duration-metric series
   * (prefix HIST_KEY_PREFIX, dimensions + histogram.dimensions) or its
   * calls-metric series (CALLS_KEY_PREFIX, dimensions + calls_dimensions); the
   * cardinality limit applies to each metric's series on their own.
   */
  _splitId(res, service, span, resAttrs, spanAttrs, status, prefix, scope = null) {
    const c = this.cfg;
    const calls = prefix === CALLS_KEY_PREFIX;
    const d = calls ? c.callsDims : c.histDims;
    const keyStr = prefix + keys.buildKeyString(service, span.name, span.kind, status, d, spanAttrs, resAttrs,
      c.exclude, scope);
    const known = res.byKey.get(keyStr);
    if (known !== undefined) return known;
    const kind = calls ? 'calls' : 'hist';
    if (c.cardinalityLimit > 0 && (res.nByKind[kind] || 0) >= c.cardinalityLimit) {
      return this._intern(res, prefix + OVERFLOW_KEY, calls ? 'calls-overflow' : 'hist-overflow', 0,
        () => [{ key: 'otel.metric.overflow', value: { type: 'bool', value: true } }]);
    }
    return this._intern(res, keyStr, kind, status, () => keys.buildAttributes(service, span.name,
      span.kind, status, d, spanAttrs, resAttrs, c.exclude, scope));
  }

  /** events.enabled: one record per span event, keyed by the span key + event dimensions. */
  _eventId(res, service, span, resAttrs, spanAttrs, event, scope = null) {
    const c = this.cfg;
    const status = span.status ? span.status.code : 0;
    const evAttrs = keys.attrMap(event.attributes);
    const base = keys.buildKeyString(service, span.name, span.kind, status, c.dims, spanAttrs,
      resAttrs, c.exclude, scope);
    const evKey = keys.buildKeyString('', '', 0, 0, c.eventDims, evAttrs, new Map(),
      new Set([keys.SERVICE_NAME_KEY, 'span.name', 'span.kind', 'status.code']));
    return this._intern(res, EVENT_KEY_PREFIX + base + evKey, 'event', status, () =>
      keys.buildAttributes(service, span.name, span.kind, status, c.dims, spanAttrs, resAttrs, c.exclude, scope)
        .concat(keys.buildAttributes('', '', 0, 0, c.eventDims, evAttrs, new Map(),
          new Set([keys.SERVICE_NAME_KEY, 'span.name', 'span.kind', 'status.code']))));
  }

  /**
   * ConsumeTraces: ExportTraceServiceRequest bytes or a decoded request
   * (otlp.js shape).  The span-name rules are applied first (a decoded
   * request's names are rewritten in place).
   */
  consumeTraces(req) {
    if (!this.handle) throw new Error('connector is shut down');
    const isBytes = Buffer.isBuffer(req) || req instanceof Uint8Array;
    if (isBytes && this.col && this._consumeNative(asBuffer(req))) return;
    this._consumeJs(isBytes ? otlp.decodeTraces(req) : req);
  }

  /**
   * Many requests at once (what the pipeline's queue hands over): byte
   * requests are columnised on the native columnizer's worker threads
   * (columnizer_threads) and committed in order, so the ids, dictionary and
   * columns are those of consumeTraces called on each in turn.  Returns one
   * entry per request: null, or the Error consumeTraces would have thrown.
   * Never throws past the first request: when the columnizer or the engine
   * fails part-way, the requests already applied keep null and only the rest
   * get the error (a sender that retries them counts nothing twice).  An
   * engine error is marked `deferred`: the engine runs asynchronously, so it
   * may come from columns of earlier requests.
   */
  consumeTracesBatch(reqs) {
    if (!this.handle) throw new Error('connector is shut down');
    const errs = new Array(reqs.length).fill(null);
    let i = 0;
    try {
      i = this._consumeBatchFrom(reqs, errs);
    } catch (e) {
      i = e.batchAt !== undefined ? e.batchAt : 0;
      for (let j = i; j < reqs.length; j++) errs[j] = e;
    }
    return errs;
  }

  /**
   * consumeTracesBatch's loop; a throw carries `batchAt`, the first request
   * not aggregated: on a columnizer failure the first one not applied, on an
   * engine failure the first one whose spans were in the failed columns (the
   * requests since the last successful drain of this batch).
   */
  _consumeBatchFrom(reqs, errs) {
    let i = 0, pendFrom = 0;
    const at = (e, k) => {
      if (e && typeof e === 'object' && e.batchAt === undefined) e.batchAt = k;
      return e;
    };
    while (i < reqs.length) {
      const isBytes = Buffer.isBuffer(reqs[i]) || reqs[i] instanceof Uint8Array;
      if (!isBytes || !this.col) {
        try { this.consumeTraces(reqs[i]); } catch (e) { errs[i] = e; }
        i += 1;
        continue;
      }
      const bufs = [];
      for (let j = i; j < reqs.length && (Buffer.isBuffer(reqs[j]) || reqs[j] instanceof Uint8Array); j++) {
        bufs.push(asBuffer(reqs[j]));
      }
      let br;
      try {
        br = this.addon.columnizeBatch(this.col, bufs);
      } catch (e) {
        throw at(e, i);
      }
      // plain requests (nothing new, status ok) have no result object: their
      // resource touches come per gap between the ones that do (touch/touchEnd)
      let t = 0, gap = 0, plainN = 0;
      const touchTo = (end) => { for (; t < end; t++) this._touchResource(br.touch[t]); };
      for (let k = 0; k < br.done; k++) {
        const r = br.results[k];
        if (r === undefined) { plainN += 1; continue; }
        touchTo(br.touchEnd[gap++]);
        try {
          if (!this._applyNative(r, bufs[k])) this._consumeJs(otlp.decodeTraces(bufs[k]));
        } catch (e) {
          errs[i + k] = e;
        }
      }
      touchTo(br.touch.length);
      this.nativeRequests += plainN;
      if (br.plainEventRecords) this.eventRecords += br.plainEventRecords;
      if (br.maxEnd > this.nativeMaxEnd) this.nativeMaxEnd = br.maxEnd;
      this.nativeBuffered = br.buffered;
      i += br.done;
      if (br.buffered >= this.cols.cap) {
        try {
          this._drain();
        } catch (e) {
          // the engine runs asynchronously: the error may also concern
          // columns of earlier batches, already acknowledged
          e.deferred = true;
          throw at(e, pendFrom);
        }
        pendFrom = i;
      }
    }
    return i;
  }

  /** The JavaScript columnizer over a decoded request. */
  _consumeJs(req) {
    this.jsRequests += 1;
    if (this.rules.length) {
      for (const rs of req.resourceSpans || []) {
        for (const ss of rs.scopeSpans || []) for (const sp of ss.spans || []) sp.name = applyRules(sp.name, this.rules);
      }
    }
    const cols = this.cols;
    for (const rs of req.resourceSpans || []) {
      const resAttrs = keys.attrMap(rs.resource && rs.resource.attributes);
      const svc = resAttrs.get(keys.SERVICE_NAME_KEY);
      if (svc === undefined) continue;  // A1: no service.name -> nothing
      const service = svc.type === 'string' ? svc.value : '';  // pcommon.Value.Str()
      const res = this._resource(resAttrs);
      const svcId = this._serviceId(service);
      for (const ss of rs.scopeSpans || []) {
        const scope = keys.includedScope(ss.scope, this.cfg.scopes);
        for (const span of ss.spans || []) {
          const spanAttrs = this.cfg.dims.length ? keys.attrMap(span.attributes) : undefined;
          const sid = this._seriesId(res, service, span, resAttrs, spanAttrs, scope);
          if (this.cfg.exemplars) this._exemplar(sid, span);
          if (this.cfg.splitKeys) {  // the calls series gets the span as a second record
            const code = span.status ? span.status.code : 0;
            this._pushCalls(this._splitId(res, service, span, resAttrs, spanAttrs, code, CALLS_KEY_PREFIX, scope), span);
          }
          const i = cols.n;
          cols.keyHash[i] = sid;
          cols.startNs[i] = BigInt.asUintN(64, BigInt(span.startTimeUnixNano || 0));
          cols.endNs[i] = BigInt.asUintN(64, BigInt(span.endTimeUnixNano || 0));
          const tid = span.traceId;
          if (tid && tid.length === 16) {
            cols.w0u8.set(tid.subarray(0, 8), 8 * i);
            cols.w1u8.set(tid.subarray(8, 16), 8 * i);
          } else {
            cols.traceW0[i] = 0n;
            cols.traceW1[i] = 0n;
          }
          const kind = span.kind >= 0 && span.kind <= 7 ? span.kind : 7;  // >5: "" either way
          const code = span.status ? span.status.code : 0;
          const st = code >= 0 && code <= 3 ? code : 3;
          cols.meta[i] = (svcId | (kind << 16) | (st << 19)) >>> 0;
          cols.n = i + 1;
          if (cols.n === cols.cap) this._drain();
          // events.enabled: the span's event records follow it (the native order)
          if (this.cfg.events && span.events && span.events.length) {
            for (const ev of span.events) this._pushEvent(this._eventId(res, service, span, resAttrs, spanAttrs, ev, scope));
          }
        }
      }
    }
  }

  /**
   * Native path: the addon columnises the request into its own buffer and
   * reports what is new (services, resources, series); the host decodes only
   * those messages to keep its dictionary, and checks that it derives the same
   * ids.  Returns false when the request needs the JavaScript path.
   */
  _consumeNative(bytes) {
    const r = this.addon.columnize(this.col, bytes);
    if (!this._applyNative(r, bytes)) return false;
    if (r.spans) {
      if (r.maxEnd > this.nativeMaxEnd) this.nativeMaxEnd = r.maxEnd;
      this.nativeBuffered = r.buffered;
      if (r.buffered >= this.cols.cap) this._drain();
    }
    return true;
  }

  /** Host bookkeeping of one native columnize result (false: fallback). */
  _applyNative(r, bytes) {
    let remapped = null;  // native -> host ids of this request's series (64-bit collisions)
    if (r.status === 'fallback') return false;
    if (r.status !== 'ok') throw new Error(`OTLP request: ${r.error}`);
    this.nativeRequests += 1;
    for (const [name, id] of r.newServices || NONE) this.services.set(name, id);
    for (const nr of r.newResources || NONE) {
      if (this._touchResource(nr.hash)) continue;  // known to the host, forgotten natively
      const attrs = nr.off >= 0 ? otlp.decodeResource(new otlp.Reader(bytes, nr.off, nr.off + nr.len)).attributes : [];
      const res = this._resource(keys.attrMap(attrs));
      if (res.hash !== nr.hash) throw new Error('native/JS resource hash mismatch');
    }
    for (const h of r.resources) this._touchResource(h);
    for (const ns of r.newSeries || NONE) {
      const res = this.resources.get(ns.resHash) || this.evicted.get(ns.resHash);
      if (!res) throw new Error('native series for an unknown resource');
      const span = otlp.decodeSpan(new otlp.Reader(bytes, ns.off, ns.off + ns.len));
      span.name = applyRules(span.name, this.rules);
      const svc = res.attributes.get(keys.SERVICE_NAME_KEY);
      const service = svc && svc.type === 'string' ? svc.value : '';
      const spanAttrs = this.cfg.dims.length ? keys.attrMap(span.attributes) : undefined;
      const resAttrs = this._spanResourceAttrs(bytes, ns, res);
      this._verifyingNative = true;
      let sid;
      try {
        sid = this._seriesId(res, service, span, resAttrs, spanAttrs);
      } finally {
        this._verifyingNative = false;
      }
      // the host dictionary decides: after a collision the two sides can differ
      // (the native side does not see series interned by a JavaScript-path request)
      if (sid !== ns.sid) {
        this.addon.columnizerRemap(this.col, ns.sid, sid);
        this.nativeRemaps += 1;
        (remapped || (remapped = new Map())).set(ns.sid, sid);
      }
    }
    for (const ne of r.newEventSeries || NONE) {  // events.enabled: verified as the JS path keys them
      const res = this.resources.get(ne.resHash) || this.evicted.get(ne.resHash);
      if (!res) throw new Error('native event series for an unknown resource');
      const span = otlp.decodeSpan(new otlp.Reader(bytes, ne.off, ne.off + ne.len));
      span.name = applyRules(span.name, this.rules);
      const svc = res.attributes.get(keys.SERVICE_NAME_KEY);
      const service = svc && svc.type === 'string' ? svc.value : '';
      const spanAttrs = this.cfg.dims.length ? keys.attrMap(span.attributes) : undefined;
      const resAttrs = this._spanResourceAttrs(bytes, ne, res);
      this._verifyingNative = true;
      let sid;
      try {
        sid = this._eventId(res, service, span, resAttrs, spanAttrs, span.events[ne.event]);
      } finally {
        this._verifyingNative = false;
      }
      if (sid !== ne.sid) {
        this.addon.columnizerRemap(this.col, ne.sid, sid);
        this.nativeRemaps += 1;
      }
    }
    if (r.eventRecords) this.eventRecords += r.eventRecords;
    for (const ex of r.exemplars || NONE) {  // exemplars.enabled: the native side's candidates, in order
      const sid = remapped && remapped.has(ex.sid) ? remapped.get(ex.sid) : ex.sid;
      if (!this.series.has(sid)) continue;
      // the native side reports the fields of a span with 16-B trace and 8-B span ids
      this._exemplar(sid, ex.traceId ? { traceId: ex.traceId, spanId: ex.spanId, startTimeUnixNano: ex.start,
        endTimeUnixNano: ex.end } : otlp.decodeSpanExemplar(new otlp.Reader(bytes, ex.off, ex.off + ex.len)));
    }
    return true;
  }

  /** exemplars.enabled: the first max_per_data_point spans of each series per export. */
  _exemplar(sid, span) {
    const s = this.series.get(sid);
    if (s.exemplars.length >= this.cfg.exemplarsMax) return;
    const st = BigInt(span.startTimeUnixNano || 0), en = BigInt(span.endTimeUnixNano || 0);
    s.exemplars.push({ traceId: span.traceId, spanId: span.spanId, timeUnixNano: en,
      asDouble: Number(en > st ? en - st : 0n) / (this.cfg.unit === 's' ? 1e9 : 1e6) });
  }

  /** One span record of series `sid` (the JavaScript columnizer's layout). */
  _pushSpan(sid, span, svcId) {
    const cols = this.cols;
    const i = cols.n;
    cols.keyHash[i] = sid;
    cols.startNs[i] = BigInt.asUintN(64, BigInt(span.startTimeUnixNano || 0));
    cols.endNs[i] = BigInt.asUintN(64, BigInt(span.endTimeUnixNano || 0));
    const tid = span.traceId;
    if (tid && tid.length === 16) {
      cols.w0u8.set(tid.subarray(0, 8), 8 * i);
      cols.w1u8.set(tid.subarray(8, 16), 8 * i);
    } else {
      cols.traceW0[i] = 0n;
      cols.traceW1[i] = 0n;
    }
    const kind = span.kind >= 0 && span.kind <= 7 ? span.kind : 7;
    const code = span.status ? span.status.code : 0;
    const st = code >= 0 && code <= 3 ? code : 3;
    cols.meta[i] = (svcId | (kind << 16) | (st << 19)) >>> 0;
    cols.n = i + 1;
    if (cols.n === cols.cap) this._drain();
  }

  /**
   * calls_dimensions / histogram.dimensions: the calls series' record of a
   * span.  It carries the span's duration (the engine counts it into the
   * series' calls) but the out-of-range service id of the event records and no
   * kind or status bits, so the sketches see each span once, through its
   * histogram series' record: its HLL raise and, for an ERROR span, its
   * count-min cells.  Counted in callsRecords (stats() takes these records
   * out of the engine's span count).
   */
  _pushCalls(sid, span) {
    const cols = this.cols;
    const i = cols.n;
    cols.keyHash[i] = sid;
    cols.startNs[i] = BigInt.asUintN(64, BigInt(span.startTimeUnixNano || 0));
    cols.endNs[i] = BigInt.asUintN(64, BigInt(span.endTimeUnixNano || 0));
    cols.traceW0[i] = 0n;
    cols.traceW1[i] = 0n;
    cols.meta[i] = 0xFFFF;
    cols.n = i + 1;
    this.callsRecords += 1;
    if (cols.n === cols.cap) this._drain();
  }

  /** An event record: counted by the engine like a span of duration 0, with an
   * out-of-range service id so it touches no sketch. */
  _pushEvent(sid) {
    const cols = this.cols;
    const i = cols.n;
    cols.keyHash[i] = sid;
    cols.startNs[i] = 0n;
    cols.endNs[i] = 0n;
    cols.traceW0[i] = 0n;
    cols.traceW1[i] = 0n;
    cols.meta[i] = 0xFFFF;
    cols.n = i + 1;
    this.eventRecords += 1;
    if (cols.n === cols.cap) this._drain();
  }

  /** Hand the buffered columns to the engine, advancing the window ring first. */
  _drain() {
    const cols = this.cols;
    if (cols.n === 0 && this.nativeBuffered === 0) return;
    let maxEnd = this.nativeBuffered ? this.nativeMaxEnd : 0n;
    for (let i = 0; i < cols.n; i++) if (cols.endNs[i] > maxEnd) maxEnd = cols.endNs[i];
    const maxWid = maxEnd / this.cfg.windowNs;
    const nw = BigInt(this.cfg.nWindows);
    if (this.windowBase === null) {
      const base = maxWid >= nw - 1n ? maxWid - (nw - 1n) : 0n;
      this.addon.windowAdvance(this.handle, base);
      this.windowBase = base;
      this.sketchWatermark = base;
    } else if (maxWid >= this.windowBase + nw) {
      const base = maxWid - nw + 1n;
      if (this.cfg.emitSketches) {  // read windows about to be retired, once
        const top = base < this.maxWindowSeen + 1n ? base : this.maxWindowSeen + 1n;
        for (let w = this.sketchWatermark > this.windowBase ? this.sketchWatermark : this.windowBase; w < top; w++) {
          this.closedWindows.push(this._readWindow(w));
        }
      }
      if (this.sketchWatermark < base) this.sketchWatermark = base;
      this.addon.windowAdvance(this.handle, base);
      this.windowBase = base;
    }
    if (maxWid > this.maxWindowSeen) this.maxWindowSeen = maxWid;
    let applied = false;
    try {
      if (cols.n) this.addon.ingest(this.handle, cols.view());
      cols.n = 0;
      if (this.nativeBuffered) this.addon.columnizerIngest(this.col);
      applied = true;
    } finally {
      // a failed ingest rejects the requests these columns hold
      // (consumeTracesBatch reports them to their senders): drop the columns,
      // JavaScript and native, so a sender's retry counts nothing twice
      cols.n = 0;
      if (!applied && this.nativeBuffered) this.addon.columnizerTake(this.col);
      this.nativeBuffered = 0;
      this.nativeMaxEnd = 0n;
    }
  }

  // ------------------------------------------------------------ export

  /**
   * exportMetrics: drain, flush the engine's delta, fold it into the host's
   * cumulative state (or emit it as delta) and build the OTLP metrics request
   * (buildMetrics).  Returns the request object; otlp.encodeMetrics() gives bytes.
   */
  exportMetrics() {
    if (!this.handle) throw new Error('connector is shut down');
    this._drain();
    const now = this.clock();
    const expo = this.cfg.expMaxSize !== 0;
    const r = expo ? this.addon.flushExp(this.handle) : this.addon.flush(this.handle);
    if (r.status === this.addon.status.EFULL) this._reportDrops();
    const nb = r.nBuckets;
    const delta = this.cfg.temporality === otlp.AGGREGATION_TEMPORALITY.DELTA;
    const touched = new Set();
    for (let i = 0; i < r.nSeries; i++) {
      const s = this.series.get(r.keyHash[i]);
      if (s === undefined) continue;  // evicted and dropped since; its delta is discarded
      if (expo) {
        // s.counts holds the series' go-expohisto state in this mode
        if (delta || s.counts === null) s.counts = expohisto.empty();
        expohisto.fold(s.counts, expohisto.fromResult(r, i), this.cfg.expMaxSize);
      } else {
        if (delta || s.counts === null) { s.counts = new Array(nb).fill(0n); s.sumNs = 0n; }
        for (let b = 0; b < nb; b++) s.counts[b] += r.bucketCounts[i * nb + b];
        s.sumNs += r.sumNs[i];
      }
      touched.add(s.sid);
    }
    const resourceMetrics = [];
    const emitResource = (res) => {
      const sids = res.sids.filter((sid) => (delta ? touched.has(sid) : this.series.get(sid).counts !== null));
      if (sids.length === 0) return;
      resourceMetrics.push({ resource: { attributes: Array.from(res.attributes, ([key, value]) => ({ key, value })) },
        scopeMetrics: [{ scope: { name: 'spanmetricsconnector' },
          metrics: this._buildMetrics(res, sids, now, delta) }] });
    };
    for (const res of this.resources.values()) emitResource(res);
    for (const res of this.evicted.values()) emitResource(res);
    // resetState: delta purges; cumulative drops what the LRU evicted and
    // (metrics_expiration) the resources not seen within the expiration
    if (!delta && this.cfg.expirationNs) {
      for (const [h, res] of [...this.resources]) {
        if (now - res.lastSeen >= this.cfg.expirationNs) {
          this.resources.delete(h);
          this.evicted.set(h, res);
        }
      }
    }
    for (const res of this.evicted.values()) {
      for (const sid of res.sids) { this.series.delete(sid); this.lastDeltaTs.delete(sid); }
      if (this.col) this.addon.columnizerForget(this.col, res.hash);
    }
    this.evicted.clear();
    if (delta) for (const sid of touched) this.series.get(sid) && (this.series.get(sid).counts = null);
    if (this.cfg.emitSketches) {
      for (let w = this.sketchWatermark; this.windowBase !== null && w < this.maxWindowSeen; w++) {
        this.closedWindows.push(this._readWindow(w));
      }
      if (this.windowBase !== null && this.sketchWatermark < this.maxWindowSeen) this.sketchWatermark = this.maxWindowSeen;
      if (this.closedWindows.length) resourceMetrics.push(this._sketchMetrics(this.closedWindows));
      this.closedWindows = [];
    }
    return { resourceMetrics };
  }

  /**
   * More distinct series in one flush interval than key_capacity: the engine
   * dropped spans (sa_flush returned SA_EFULL).  Counted (droppedFlushes,
   * droppedSpans in stats()) and reported through `onDrop` (default: a warning
   * on stderr, at most once a minute) -- never silent.  The engine reclaims
   * its key table at flush time, so the series of earlier intervals do not
   * fill it; only one interval's series have to fit.
   */
  _reportDrops() {
    this.droppedFlushes += 1;
    const st = this.addon.stats(this.handle);
    const dropped = st.droppedTableFull !== undefined ? BigInt(st.droppedTableFull) : 0n;
    const info = { droppedSpans: dropped, keyCapacity: this.cfg.keyCapacity, droppedFlushes: this.droppedFlushes };
    this.droppedSpans = dropped;
    if (this.onDrop) return this.onDrop(info);
    const now = Date.now();
    if (!this._lastDropWarn || now - this._lastDropWarn > 60000) {
      this._lastDropWarn = now;
      process.emitWarning(`spanmetrics: ${dropped} spans dropped so far: more series in one flush interval ` +
        `than key_capacity (${this.cfg.keyCapacity})`, 'SpanMetricsDropWarning');
    }
    return undefined;
  }

  _buildMetrics(res, sids, now, delta) {
    const c = this.cfg;
    const ns = c.namespace ? c.namespace + '.' : '';
    const temporality = c.temporality;
    const div = c.unit === 's' ? 1e9 : 1e6;
    const calls = [], hists = [], events = [];
    for (const sid of sids) {
      const s = this.series.get(sid);
      let start = res.startTs;
      if (delta) {
        const last = this.lastDeltaTs.get(sid);
        if (last !== undefined) start = last;
        this.lastDeltaTs.set(sid, now);
      }
      const e = c.expMaxSize ? s.counts : null;
      let count = 0n;
      if (e) count = e.count;
      else for (const x of s.counts) count += x;
      if (s.kind === 'event') {
        events.push({ attributes: s.dpAttrs, startTimeUnixNano: start, timeUnixNano: now, asInt: count });
        continue;
      }
      // (split keys: a 'calls' series feeds only the calls metric, a 'hist'
      // series only the duration metric)
      const isCalls = s.kind === 'calls' || s.kind === 'calls-overflow';
      const isHist = s.kind === 'hist' || s.kind === 'hist-overflow';
      if (!isHist) calls.push({ attributes: s.dpAttrs, startTimeUnixNano: start, timeUnixNano: now, asInt: count });
      if (isCalls || c.histogramDisable) {
        s.exemplars = [];
        continue;
      }
      const h = e
        ? { attributes: s.dpAttrs, startTimeUnixNano: start, timeUnixNano: now, count, sum: Number(e.sumNs) / div,
          scale: e.scale, zeroCount: e.zeroCount, positive: { offset: e.offset, bucketCounts: e.counts.slice() },
          ...(count ? { min: e.min, max: e.max } : {}) }
        : { attributes: s.dpAttrs, startTimeUnixNano: start, timeUnixNano: now, count,
          sum: Number(s.sumNs) / div, bucketCounts: s.counts.slice(), explicitBounds: c.bounds };
      if (s.exemplars.length) h.exemplars = s.exemplars;
      hists.push(h);
      s.exemplars = [];  // exemplars cover one export interval, both temporalities
    }
    if (this.col && c.exemplars && this.addon.columnizerResetExemplars) this.addon.columnizerResetExemplars(this.col);
    const out = [
      { name: ns + 'calls', sum: { dataPoints: calls, aggregationTemporality: temporality, isMonotonic: true } }];
    if (!c.histogramDisable) {
      out.push(c.expMaxSize
        ? { name: ns + 'duration', unit: c.unit,
          exponentialHistogram: { dataPoints: hists, aggregationTemporality: temporality } }
        : { name: ns + 'duration', unit: c.unit, histogram: { dataPoints: hists, aggregationTemporality: temporality } });
    }
    if (c.events) {
      out.push({ name: ns + 'events', sum: { dataPoints: events, aggregationTemporality: temporality,
        isMonotonic: true } });
    }
    return out;
  }

  // ------------------------------------------------------------ sketches

  /**
   * Sketches of one resident window: distinct traces per service (HLL) and a
   * count-min point query of ERROR spans per series.
   */
  windowSketch(windowId) {
    if (!this.handle) throw new Error('connector is shut down');
    this._drain();
    return this._readWindow(windowId);
  }

  _readWindow(windowId) {
    const w = this.addon.windowRead(this.handle, BigInt(windowId));
    const m = 1 << w.hllP;
    const distinct = new Map();
    for (const [name, id] of this.services) {
      if (id < w.nServices) distinct.set(name, this.addon.hllEstimate(w.hll.subarray(id * m, (id + 1) * m), w.hllP));
    }
    const shift = 64n - BigInt(Math.log2(w.cmsW));
    const errorCount = (sid) => {
      let best = 0xFFFFFFFF;
      for (let j = 0; j < w.cmsD; j++) {
        const col = Number(splitmix64(BigInt.asUintN(64, sid) ^ CMS_SEED[j]) >> shift);
        best = Math.min(best, w.cms[j * w.cmsW + col]);
      }
      return best;
    };
    const topErrors = (k = this.cfg.topK) => {
      const out = [];
      for (const s of this.series.values()) {
        // the series whose records carry the span's status: never a calls-only
        // or event series (their records touch no sketch)
        if (s.status !== 2 || !SKETCH_KINDS.has(s.kind)) continue;
        const n = errorCount(s.sid);
        if (n > 0) out.push({ sid: s.sid, key: s.keyStr, attributes: s.dpAttrs, errors: n });
      }
      out.sort((a, b) => b.errors - a.errors);
      return out.slice(0, k);
    };
    return { windowId: w.windowId, startNs: w.windowId * this.cfg.windowNs, distinct, errorCount,
      topErrors, raw: w };
  }

  _sketchMetrics(windows) {
    const ns = this.cfg.namespace ? this.cfg.namespace + '.' : '';
    const distinct = [], errors = [];
    for (const w of windows) {
      const t0 = w.startNs, t1 = w.startNs + this.cfg.windowNs;
      for (const [name, est] of w.distinct) {
        if (est === 0) continue;
        distinct.push({ attributes: [{ key: keys.SERVICE_NAME_KEY, value: { type: 'string', value: name } }],
          startTimeUnixNano: t0, timeUnixNano: t1, asDouble: est });
      }
      for (const e of w.topErrors()) {
        errors.push({ attributes: e.attributes, startTimeUnixNano: t0, timeUnixNano: t1, asInt: BigInt(e.errors) });
      }
    }
    return { resource: { attributes: [] }, scopeMetrics: [{ scope: { name: 'spanmetricsconnector' }, metrics: [
      { name: ns + 'window.distinct_traces', gauge: { dataPoints: distinct } },
      { name: ns + 'window.errors', gauge: { dataPoints: errors } }] }] };
  }

  stats() {
    const s = this.addon.stats(this.handle);
    // the engine counts records: a span's own, plus the auxiliary ones (event
    // records, split keys' calls records), which carry service id 0xFFFF
    const aux = BigInt(this.eventRecords + this.callsRecords);
    if (typeof s.spans === 'bigint') s.records = s.spans, s.spans -= aux;
    if (typeof s.invalidService === 'bigint') s.invalidService -= aux;
    return Object.assign(s, { callsRecords: this.callsRecords, resources: this.resources.size, series: this.series.size,
      services: this.services.size, droppedFlushes: this.droppedFlushes, droppedSpans: this.droppedSpans,
      collisions: this.collisions,
      eventRecords: this.eventRecords, nativeRequests: this.nativeRequests, jsRequests: this.jsRequests,
      nativeRemaps: this.nativeRemaps });
  }
}

module.exports = { SpanMetricsConnector, normalizeConfig, parseDurationNs, splitmix64, Columns };
