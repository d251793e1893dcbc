'use strict';
/**
 * Loads the in-tree N-API addon (build/spanagg.node, built by `make -C
 * host/node` or __graft_entry__.build()).  There is no JS fallback for the
 * aggregation: a missing addon is an error, never a silent CPU path.
 */
const path = require('path');

const ADDON_PATH = path.resolve(__dirname, '..', 'build', 'spanagg.node');
let cached = null;

function load() {
  if (cached) return cached;
  try {
    cached = require(ADDON_PATH);
  } catch (err) {
    const e = new Error(`spanagg N-API addon not loadable from ${ADDON_PATH} ` +
      `(build it with \`make -C host/node\`): ${err.message}`);
    e.cause = err;
    throw e;
  }
  if (typeof cached.xxh64 === 'function') require('./keys').useNativeXxh64(cached.xxh64);
  return cached;
}

module.exports = { load, ADDON_PATH };
