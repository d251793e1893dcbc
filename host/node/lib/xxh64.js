'use strict';
/**
 * xxHash64 (seed 0/1) in BigInt arithmetic -- the hash the connector's key
 * identity uses ([UPSTREAM] cespare/xxhash/v2, via pdatautil.MapHash) and that
 * spanagg/keys.py (Python, `xxhash` package) uses for series ids.  Checked
 * against keys.py-generated vectors in test/test_host.js.
 */
const M64 = (1n << 64n) - 1n;
const P1 = 0x9E3779B185EBCA87n;
const P2 = 0xC2B2AE3D27D4EB4Fn;
const P3 = 0x165667B19E3779F9n;
const P4 = 0x85EBCA77C2B2AE63n;
const P5 = 0x27D4EB2F165667C5n;

const rotl = (x, r) => ((x << BigInt(r)) | (x >> BigInt(64 - r))) & M64;
const mul = (a, b) => (a * b) & M64;
const round = (acc, lane) => mul(rotl((acc + mul(lane, P2)) & M64, 31), P1);
const merge = (acc, v) => ((mul((acc ^ round(0n, v)), P1) + P4) & M64);

function readU64(b, i) {
  let x = 0n;
  for (let k = 7; k >= 0; --k) x = (x << 8n) | BigInt(b[i + k]);
  return x;
}
function readU32(b, i) {
  return BigInt((b[i] | (b[i + 1] << 8) | (b[i + 2] << 16) | (b[i + 3] << 24)) >>> 0);
}

/** xxh64 of a Uint8Array (or Buffer) with a BigInt/number seed; returns BigInt. */
function xxh64(bytes, seed = 0n) {
  seed = BigInt(seed) & M64;
  const n = bytes.length;
  let i = 0;
  let h;
  if (n >= 32) {
    let v1 = (seed + P1 + P2) & M64, v2 = (seed + P2) & M64, v3 = seed, v4 = (seed - P1) & M64;
    for (; i + 32 <= n; i += 32) {
      v1 = round(v1, readU64(bytes, i));
      v2 = round(v2, readU64(bytes, i + 8));
      v3 = round(v3, readU64(bytes, i + 16));
      v4 = round(v4, readU64(bytes, i + 24));
    }
    h = (rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18)) & M64;
    h = merge(h, v1); h = merge(h, v2); h = merge(h, v3); h = merge(h, v4);
  } else {
    h = (seed + P5) & M64;
  }
  h = (h + BigInt(n)) & M64;
  for (; i + 8 <= n; i += 8) {
    h ^= round(0n, readU64(bytes, i));
    h = (mul(rotl(h, 27), P1) + P4) & M64;
  }
  if (i + 4 <= n) {
    h ^= mul(readU32(bytes, i), P1);
    h = (mul(rotl(h, 23), P2) + P3) & M64;
    i += 4;
  }
  for (; i < n; ++i) {
    h ^= mul(BigInt(bytes[i]), P5);
    h = mul(rotl(h, 11), P1);
  }
  h ^= h >> 33n; h = mul(h, P2);
  h ^= h >> 29n; h = mul(h, P3);
  h ^= h >> 32n;
  return h;
}

module.exports = { xxh64 };
