'use strict';
/**
 * TEST-ONLY stand-in for build/spanagg.node, so the connector's host logic
 * (resources, temporality, LRU, window bookkeeping) is testable without a GPU.
 * It is never loaded by lib/: the product path requires the real addon
 * (lib/addon.js throws when it is missing).  Aggregation here is a plain
 * restatement of the engine contract (include/spanagg.h): integer-threshold
 * buckets, exact ns sums, per-service HLL, count-min over ERROR spans.
 */
const { xxh64 } = require('../lib/xxh64');
const { splitmix64 } = require('../lib/connector');
const { Histogram } = require('./expo_ref');

const DEFAULT_BOUNDS = [2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000];
const CMS_SEED = [0x9E3779B97F4A7C15n, 0xBF58476D1CE4E5B9n, 0x94D049BB133111EBn,
  0xD6E8FEB86659FD93n, 0xA0761D6478BD642Fn, 0xE7037ED1A0B428DBn, 0x8EBC6AF09C88C6E3n,
  0x589965CC75374CC3n];

class FakeAddon {
  constructor() {
    this.status = { OK: 0, EINVAL: -1, ENOMEM: -2, EDEVICE: -3, EFULL: -4, ERANGE: -5, ESTATE: -6 };
    this.batches = [];
    this.base = 0n;
  }
  abiVersion() { return 3; }
  configDefault() {
    return { bounds: DEFAULT_BOUNDS.slice(), unit: 'ms', hllP: 14, cmsD: 4, cmsW: 2048,
      windowNs: 10000000000n, nWindows: 8, nServices: 64, keyCapacity: 1000, device: 0, flags: 0 };
  }
  hllEstimate(regs, p) {
    const m = 1 << p;
    let sum = 0, zeros = 0;
    for (let j = 0; j < m; j++) { sum += Math.pow(2, -regs[j]); zeros += regs[j] === 0; }
    const alpha = m === 16 ? 0.673 : m === 32 ? 0.697 : m === 64 ? 0.709 : 0.7213 / (1 + 1.079 / m);
    let e = alpha * m * m / sum;
    if (e <= 2.5 * m && zeros !== 0) e = m * Math.log(m / zeros);
    return e;
  }
  create(cfg) {
    this.cfg = cfg;
    this.div = cfg.unit === 's' ? 1e9 : 1e6;
    this.red = new Map();
    this.windows = new Map();
    return { fake: true };
  }
  destroy() { this.cfg = null; }
  _bucket(d) {
    const x = d / this.div;
    let i = 0;
    while (i < this.cfg.bounds.length && this.cfg.bounds[i] < x) i++;
    return i;
  }
  _window(wid) {
    let w = this.windows.get(wid);
    if (!w) {
      w = { hll: new Uint8Array(this.cfg.nServices << this.cfg.hllP),
        cms: new Uint32Array(this.cfg.cmsD * this.cfg.cmsW) };
      this.windows.set(wid, w);
    }
    return w;
  }
  ingest(h, b) {
    const copy = {};
    for (const k of Object.keys(b)) copy[k] = b[k].slice();
    this.batches.push(copy);
    const nb = this.cfg.bounds.length + 1;
    const p = this.cfg.hllP;
    this.nRecords = (this.nRecords || 0n) + BigInt(b.keyHash.length);
    for (let i = 0; i < b.keyHash.length; i++) {
      const sid = b.keyHash[i];
      if ((b.meta[i] & 0xFFFF) >= this.cfg.nServices) this.nInvalid = (this.nInvalid || 0n) + 1n;
      const d = b.endNs[i] > b.startNs[i] ? b.endNs[i] - b.startNs[i] : 0n;
      let r = this.red.get(sid);
      if (!r) {
        r = { counts: new Array(nb).fill(0n), sumNs: 0n, expo: new Histogram(this.cfg.expMaxSize || 160),
          minNs: 0n, maxNs: 0n };
        this.red.set(sid, r);
      }
      r.counts[this._bucket(Number(d))] += 1n;
      if (r.expo.count === 0n || d < r.minNs) r.minNs = d;
      if (r.expo.count === 0n || d > r.maxNs) r.maxNs = d;
      r.expo.update(Number(d) / this.div);
      r.sumNs += d;
      const svc = b.meta[i] & 0xFFFF, status = (b.meta[i] >>> 19) & 3;
      const wid = b.endNs[i] / this.cfg.windowNs;
      if (svc >= this.cfg.nServices || wid < this.base || wid >= this.base + BigInt(this.cfg.nWindows)) continue;
      const w = this._window(wid);
      const tid = Buffer.alloc(16);
      tid.writeBigUInt64LE(b.traceW0[i], 0);
      tid.writeBigUInt64LE(b.traceW1[i], 8);
      const x = xxh64(tid, 0n);
      const idx = Number(x >> BigInt(64 - p));
      const rest = ((x << BigInt(p)) | (1n << BigInt(p - 1))) & ((1n << 64n) - 1n);
      const rho = 65 - rest.toString(2).length;
      const reg = (svc << p) + idx;
      if (w.hll[reg] < rho) w.hll[reg] = rho;
      if (status === 2) {
        const shift = 64n - BigInt(Math.log2(this.cfg.cmsW));
        for (let j = 0; j < this.cfg.cmsD; j++) {
          const col = Number(splitmix64(sid ^ CMS_SEED[j]) >> shift);
          w.cms[j * this.cfg.cmsW + col] += 1;
        }
      }
    }
  }
  flush() {
    const keysSorted = [...this.red.keys()].sort((a, b) => (a < b ? -1 : a > b ? 1 : 0));
    const nb = this.cfg.bounds.length + 1, n = keysSorted.length;
    const out = { status: 0, nSeries: n, nBuckets: nb, keyHash: new BigUint64Array(keysSorted),
      bucketCounts: new BigUint64Array(n * nb), calls: new BigUint64Array(n),
      sumNs: new BigUint64Array(n), sum: new Float64Array(n) };
    keysSorted.forEach((k, i) => {
      const r = this.red.get(k);
      r.counts.forEach((c, j) => { out.bucketCounts[i * nb + j] = c; out.calls[i] += c; });
      out.sumNs[i] = r.sumNs;
      out.sum[i] = Number(r.sumNs) / this.div;
    });
    this.red.clear();
    return out;
  }
  flushExp() {
    if (!this.cfg.expMaxSize) {
      const e = new Error('sa_flush_exp: engine built for explicit buckets');
      e.code = this.status.ESTATE;
      throw e;
    }
    const keysSorted = [...this.red.keys()].sort((a, b) => (a < b ? -1 : a > b ? 1 : 0));
    const m = this.cfg.expMaxSize, n = keysSorted.length;
    const out = { status: 0, nSeries: n, maxSize: m, keyHash: new BigUint64Array(keysSorted),
      count: new BigUint64Array(n), zeroCount: new BigUint64Array(n), sumNs: new BigUint64Array(n),
      sum: new Float64Array(n), min: new Float64Array(n), max: new Float64Array(n), scale: new Int32Array(n),
      offset: new Int32Array(n), nBuckets: new Uint32Array(n), bucketCounts: new BigUint64Array(n * m) };
    keysSorted.forEach((k, i) => {
      const r = this.red.get(k), h = r.expo, b = h.buckets();
      out.count[i] = h.count; out.zeroCount[i] = h.zero; out.sumNs[i] = r.sumNs;
      out.sum[i] = Number(r.sumNs) / this.div;
      out.min[i] = Number(r.minNs) / this.div; out.max[i] = Number(r.maxNs) / this.div;
      out.scale[i] = h.scale; out.offset[i] = b.offset; out.nBuckets[i] = b.counts.length;
      b.counts.forEach((c, j) => { out.bucketCounts[i * m + j] = c; });
    });
    this.red.clear();
    return out;
  }
  windowRead(h, wid) {
    if (wid < this.base || wid >= this.base + BigInt(this.cfg.nWindows)) {
      const e = new Error('sa_window_read: window outside the resident ring');
      e.code = this.status.ERANGE;
      throw e;
    }
    const w = this._window(wid);
    return { windowId: wid, nServices: this.cfg.nServices, hllP: this.cfg.hllP, hll: w.hll.slice(),
      cmsD: this.cfg.cmsD, cmsW: this.cfg.cmsW, cms: w.cms.slice() };
  }
  windowAdvance(h, base) {
    for (const wid of [...this.windows.keys()]) if (wid < base) this.windows.delete(wid);
    this.base = base;
  }
  stats() {
    return { spans: this.nRecords || 0n, invalidService: this.nInvalid || 0n, droppedTableFull: this.dropped || 0n };
  }
}

/**
 * FakeAddon plus the REAL native columnizer of build/spanagg.node (it needs no
 * GPU): requests are columnised natively and the columns handed to the fake
 * engine, so native and JavaScript columnising can be compared on CPU.
 */
class NativeColumnizerFakeAddon extends FakeAddon {
  constructor() {
    super();
    this.real = require('../lib/addon').load();
  }
  createColumnizer(h, opts) {
    return this.real.createColumnizer(null, Object.assign({}, opts, this.collide ? { testCollideSeed0: true } : {},
      this.batched ? { testBatched: true } : {}));
  }
  columnize(c, bytes) { return this.real.columnize(c, bytes); }
  columnizeBatch(c, bufs) { return this.real.columnizeBatch(c, bufs); }
  columnizerServiceId(c, name) { return this.real.columnizerServiceId(c, name); }
  columnizerForget(c, h) { return this.real.columnizerForget(c, h); }
  columnizerLearn(c, h, key, sid) { return this.real.columnizerLearn(c, h, key, sid); }
  columnizerRemap(c, from, to) { return this.real.columnizerRemap(c, from, to); }
  columnizerResetExemplars(c) { return this.real.columnizerResetExemplars(c); }
  columnizerDestroy(c) { return this.real.columnizerDestroy(c); }
  columnizerTake(c) { return this.real.columnizerTake(c); }
  columnizerIngest(c) {
    const b = this.real.columnizerTake(c);
    this.ingest(null, b);
    return b.keyHash.length;
  }
}

module.exports = { FakeAddon, NativeColumnizerFakeAddon };
