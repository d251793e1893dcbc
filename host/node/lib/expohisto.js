'use strict';
/**
 * Host-side state of the connector's exponential histograms
 * (`histogram.exponential`, [UPSTREAM] spanmetricsconnector v0.125.0
 * internal/metrics exponentialHistogram -> go-expohisto
 * structure.Histogram[float64]).
 *
 * The engine (sa_flush_exp) returns each series' delta histogram for one flush
 * interval.  Cumulative temporality keeps one histogram per series for the
 * connector's lifetime (Go never resets it), so the host folds each delta into
 * it here.  go-expohisto's final state depends only on the multiset of values:
 * scale = the largest scale <= 20 at which [index(minpos), index(maxpos)] spans
 * fewer than max_size buckets, and index(v) at scale s is index(v) at scale
 * s+k shifted right by k.  Folding therefore downscales both operands to the
 * smaller scale, widens the range to the union and downscales again by the
 * least shift that fits (go-expohisto changeScale) -- the histogram Go would
 * hold after observing both intervals' values one by one.
 */

const MAX_SCALE = 20;

/** go-expohisto changeScale: least shift with (high >> c) - (low >> c) < maxSize. */
function changeScale(high, low, maxSize) {
  let c = 0;
  while (high - low >= maxSize) { high >>= 1; low >>= 1; c++; }
  return c;
}

/** Empty histogram (no observations). */
function empty() {
  return { count: 0n, zeroCount: 0n, sumNs: 0n, min: 0, max: 0, scale: MAX_SCALE, offset: 0, counts: [] };
}

/** Row i of a flushExp() result as a histogram. */
function fromResult(r, i) {
  const m = r.maxSize, nb = r.nBuckets[i];
  const counts = new Array(nb);
  for (let b = 0; b < nb; b++) counts[b] = r.bucketCounts[i * m + b];
  return { count: r.count[i], zeroCount: r.zeroCount[i], sumNs: r.sumNs[i], min: r.min[i], max: r.max[i],
    scale: r.scale[i], offset: r.offset[i], counts };
}

/** Fold delta `d` into `acc` (in place); both built with the same maxSize. */
function fold(acc, d, maxSize) {
  if (d.count === 0n) return acc;
  if (acc.count === 0n) {
    acc.min = d.min;
    acc.max = d.max;
  } else {
    acc.min = Math.min(acc.min, d.min);
    acc.max = Math.max(acc.max, d.max);
  }
  acc.count += d.count;
  acc.zeroCount += d.zeroCount;
  acc.sumNs += d.sumNs;
  if (d.counts.length === 0) return acc;
  if (acc.counts.length === 0) {
    acc.scale = d.scale;
    acc.offset = d.offset;
    acc.counts = d.counts.slice();
    return acc;
  }
  let s = Math.min(acc.scale, d.scale);
  const ka = acc.scale - s, kd = d.scale - s;
  let lo = Math.min(acc.offset >> ka, d.offset >> kd);
  let hi = Math.max((acc.offset + acc.counts.length - 1) >> ka, (d.offset + d.counts.length - 1) >> kd);
  const c = changeScale(hi, lo, maxSize);
  s -= c;
  lo >>= c;
  hi >>= c;
  const out = new Array(hi - lo + 1).fill(0n);
  for (const [h, k] of [[acc, ka + c], [d, kd + c]]) {
    for (let j = 0; j < h.counts.length; j++) out[((h.offset + j) >> k) - lo] += h.counts[j];
  }
  acc.scale = s;
  acc.offset = lo;
  acc.counts = out;
  return acc;
}

module.exports = { MAX_SCALE, changeScale, empty, fromResult, fold };
