'use strict';
/**
 * TEST-ONLY restatement of go-expohisto for the fake engine and the connector
 * tests (same algorithm as tests/golden/gen_expo.py, whose known answers
 * run.js checks this file against): Go's math.Log, the logarithm / exponent
 * index mappings and Histogram.Update one value at a time.  JavaScript
 * doubles are IEEE binary64 with no contraction, so the bits are Go's.
 */
const LN2HI = 6.93147180369123816490e-01, LN2LO = 1.90821492927058770002e-10;
const L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01;
const L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
const L7 = 1.479819860511658591e-01;
const LOG2E = 1.4426950408889634;
const dv = new DataView(new ArrayBuffer(8));

function bits(x) { dv.setFloat64(0, x); return dv.getBigUint64(0); }
function fromBits(b) { dv.setBigUint64(0, b); return dv.getFloat64(0); }

/** Go math.Frexp for normal positive x (the values this path sees). */
function frexp(x) {
  const b = bits(x);
  const e = Number((b >> 52n) & 0x7FFn);
  if (e === 0) { const [f, k] = frexp(x * 2 ** 52); return [f, k - 52]; }
  return [fromBits((b & ~(0x7FFn << 52n)) | (1022n << 52n)), e - 1022];
}

function goLog(x) {
  let [f1, ki] = frexp(x);
  if (f1 < Math.SQRT2 / 2) { f1 *= 2; ki -= 1; }
  const f = f1 - 1, k = ki;
  const s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const R = t1 + t2, hfsq = 0.5 * f * f;
  return k * LN2HI - ((hfsq - (s * (hfsq + R) + k * LN2LO)) - f);
}

function mapToIndex(v, scale) {
  const b = bits(v);
  let rawExp = Number((b >> 52n) & 0x7FFn);
  const sig = b & ((1n << 52n) - 1n);
  if (scale > 0) {
    if (v <= 2 ** -1022) return -1022 * 2 ** scale;
    if (sig === 0n) return (rawExp - 1023) * 2 ** scale - 1;
    const idx = Math.floor(goLog(v) * (LOG2E * 2 ** scale));
    return Math.min(idx, 1024 * 2 ** scale - 1);
  }
  if (rawExp === 0) rawExp -= (64 - sig.toString(2).length) - 12;
  return (rawExp - 1023 + (sig === 0n ? -1 : 0)) >> -scale;
}

class Histogram {
  constructor(maxSize) {
    this.maxSize = maxSize; this.scale = 20; this.count = 0n; this.zero = 0n; this.sum = 0;
    this.min = 0; this.max = 0; this.start = null; this.end = null; this.counts = new Map();
  }
  _changeScale(high, low) {
    let c = 0;
    while (high - low >= this.maxSize) { high >>= 1; low >>= 1; c++; }
    return c;
  }
  _downscale(c) {
    if (c <= 0) return;
    const m = new Map();
    for (const [i, n] of this.counts) m.set(i >> c, (m.get(i >> c) || 0n) + n);
    this.counts = m; this.start >>= c; this.end >>= c; this.scale -= c;
  }
  _increment(i) {
    if (this.start === null) { this.start = this.end = i; } else if (i < this.start) {
      if (this.end - i >= this.maxSize) return [this.end, i];
      this.start = i;
    } else if (i > this.end) {
      if (i - this.start >= this.maxSize) return [i, this.start];
      this.end = i;
    }
    this.counts.set(i, (this.counts.get(i) || 0n) + 1n);
    return null;
  }
  update(v) {
    if (this.count === 0n) { this.min = this.max = v; } else { this.min = Math.min(this.min, v); this.max = Math.max(this.max, v); }
    this.count += 1n;
    if (v === 0) { this.zero += 1n; return; }
    this.sum += v;
    const hl = this._increment(mapToIndex(v, this.scale));
    if (hl) {
      this._downscale(this._changeScale(hl[0], hl[1]));
      if (this._increment(mapToIndex(v, this.scale))) throw new Error('expohisto: downscale did not fit');
    }
  }
  buckets() {
    if (this.start === null) return { offset: 0, counts: [] };
    const out = [];
    for (let i = this.start; i <= this.end; i++) out.push(this.counts.get(i) || 0n);
    return { offset: this.start, counts: out };
  }
}

module.exports = { goLog, mapToIndex, Histogram };
