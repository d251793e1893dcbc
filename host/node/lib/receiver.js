'use strict';
/**
 * OTLP trace receiver, metrics exporter and memory limiter for the Node host:
 * the pieces of the demo collector's traces pipeline around the connector
 * (/root/reference/src/otel-collector/otelcol-config.yml):
 *
 *   receivers.otlp.protocols.grpc / http (:4-14)   OtlpReceiver (gRPC over h2c, HTTP/1.1)
 *   processors.memory_limiter (:101-104)           MemoryLimiter (refuses data over the soft limit)
 *   exporters.otlphttp/prometheus (:89-92)         OtlpHttpExporter (POST {endpoint}/v1/metrics)
 *
 * Only protobuf payloads are accepted (OTLP/JSON requests get 415); gzip
 * request bodies are inflated.  Responses are empty Export*ServiceResponse
 * messages.  Errors from the consumer map to HTTP 500 / gRPC INTERNAL; a
 * memory-limiter refusal maps to HTTP 503 / gRPC UNAVAILABLE, which OTLP
 * clients retry.
 */
const http = require('http');
const http2 = require('http2');
const os = require('os');
const zlib = require('zlib');

const TRACE_EXPORT_PATH = '/opentelemetry.proto.collector.trace.v1.TraceService/Export';
const GRPC_OK = 0, GRPC_INTERNAL = 13, GRPC_UNAVAILABLE = 14, GRPC_UNIMPLEMENTED = 12,
  GRPC_INVALID_ARGUMENT = 3, GRPC_RESOURCE_EXHAUSTED = 8;

class RefusedError extends Error {
  constructor(msg) { super(msg); this.refused = true; }
}

/**
 * memory_limiter: limit = limit_percentage of total memory (or limit_mib),
 * soft limit = limit - spike.  check() throws RefusedError while the process
 * RSS is above the soft limit; the demo config is 80% / 25%.
 */
class MemoryLimiter {
  constructor({ limit_percentage = 80, spike_limit_percentage = 25, limit_mib, spike_limit_mib,
    check_interval_ms = 5000, total = os.totalmem(), usage = () => process.memoryUsage().rss } = {}) {
    const limit = limit_mib !== undefined ? limit_mib * 1048576 : total * limit_percentage / 100;
    const spike = spike_limit_mib !== undefined ? spike_limit_mib * 1048576 : total * spike_limit_percentage / 100;
    this.limit = limit;
    this.soft = limit - spike;
    this.usage = usage;
    this.interval = check_interval_ms;
    this.lastCheck = -Infinity;
    this.refusing = false;
    this.refused = 0;
  }

  check(now = Date.now()) {
    if (now - this.lastCheck >= this.interval) {
      this.lastCheck = now;
      const u = this.usage();
      this.refusing = u > this.soft;
      if (u > this.limit && global.gc) global.gc();
    }
    if (this.refusing) {
      this.refused += 1;
      throw new RefusedError('data refused due to high memory usage');
    }
  }
}

/**
 * Request bodies are limited after decompression too (Go's confighttp applies
 * max_request_body_size to the decompressed body, gRPC its max_recv_msg_size
 * to the decompressed message): a small gzip bomb fails with tooLarge.
 */
function inflate(body, encoding, max = Infinity) {
  if (!encoding || encoding === 'identity') return body;
  const opts = Number.isFinite(max) ? { maxOutputLength: max } : {};
  try {
    if (encoding === 'gzip') return zlib.gunzipSync(body, opts);
    if (encoding === 'deflate') return zlib.inflateSync(body, opts);
  } catch (e) {
    const err = new Error(e instanceof RangeError || e.code === 'ERR_BUFFER_TOO_LARGE'
      ? 'decompressed request body too large' : `bad ${encoding} body: ${e.message}`);
    if (e instanceof RangeError || e.code === 'ERR_BUFFER_TOO_LARGE') err.tooLarge = true;
    else err.badRequest = true;
    throw err;
  }
  const err = new Error(`unsupported content encoding ${encoding}`);
  err.badRequest = true;
  throw err;
}

/** Errors that mean the request itself is malformed (-> 400 / INVALID_ARGUMENT). */
function isBadRequest(e) {
  return !!(e && (e.badRequest || /^(OTLP request|protobuf)/.test(String(e.message))));
}

/**
 * OTLP/gRPC + OTLP/HTTP trace receiver.  onTraces(bytes) receives the raw
 * ExportTraceServiceRequest; it may throw (RefusedError -> retryable).
 */
class OtlpReceiver {
  constructor({ host = '127.0.0.1', httpPort = 4318, grpcPort = 4317, onTraces,
    maxBodyBytes = 64 * 1048576 } = {}) {
    this.host = host;
    this.httpPort = httpPort;
    this.grpcPort = grpcPort;
    this.onTraces = onTraces;
    this.maxBody = maxBodyBytes;
    this.httpServer = null;
    this.grpcServer = null;
    this.sessions = new Set();
  }

  async start() {
    if (this.httpPort !== null) {
      this.httpServer = http.createServer((req, res) => this._http(req, res));
      await listen(this.httpServer, this.httpPort, this.host);
      this.httpPort = this.httpServer.address().port;
    }
    if (this.grpcPort !== null) {
      this.grpcServer = http2.createServer();
      this.grpcServer.on('session', (s) => { this.sessions.add(s); s.on('close', () => this.sessions.delete(s)); });
      this.grpcServer.on('stream', (stream, headers) => this._grpc(stream, headers));
      await listen(this.grpcServer, this.grpcPort, this.host);
      this.grpcPort = this.grpcServer.address().port;
    }
    return this;
  }

  async close() {
    for (const s of this.sessions) s.destroy();
    await Promise.all([this.httpServer, this.grpcServer].filter(Boolean)
      .map((srv) => new Promise((r) => srv.close(() => r()))));
  }

  _http(req, res) {
    const reply = (code, body = Buffer.alloc(0), type = 'application/x-protobuf') => {
      res.writeHead(code, { 'Content-Type': type, 'Content-Length': body.length });
      res.end(body);
    };
    if (req.method !== 'POST' || req.url.split('?')[0] !== '/v1/traces') return void (req.resume(), reply(404));
    const type = (req.headers['content-type'] || '').split(';')[0].trim();
    if (type !== 'application/x-protobuf') return void (req.resume(), reply(415, Buffer.from('only application/x-protobuf is supported'), 'text/plain'));
    readBody(req, this.maxBody).then((raw) => {
      // onTraces may return a promise (the pipeline's queue): reply once it settles
      Promise.resolve().then(() => this.onTraces(inflate(raw, req.headers['content-encoding'], this.maxBody)))
        .then(() => reply(200), (e) => {  // 200: empty ExportTraceServiceResponse
          const code = e.refused ? 503 : e.tooLarge ? 413 : isBadRequest(e) ? 400 : 500;
          reply(code, Buffer.from(String(e.message)), 'text/plain');
        });
    }, (e) => reply(e.tooLarge ? 413 : 400, Buffer.from(String(e.message)), 'text/plain'));
  }

  _grpc(stream, headers) {
    const done = (status, msg, body) => {
      if (stream.destroyed) return;
      if (!stream.headersSent) stream.respond({ ':status': 200, 'content-type': 'application/grpc' }, { waitForTrailers: true });
      stream.on('wantTrailers', () => {
        const t = { 'grpc-status': String(status) };
        if (msg) t['grpc-message'] = encodeURIComponent(msg);
        stream.sendTrailers(t);
      });
      stream.end(body || Buffer.alloc(0));
    };
    if (headers[':path'] !== TRACE_EXPORT_PATH) {
      stream.resume();
      return done(GRPC_UNIMPLEMENTED, `unknown method ${headers[':path']}`);
    }
    readBody(stream, this.maxBody).then((raw) => {
      let msgs;
      try {
        msgs = grpcUnframe(raw, headers['grpc-encoding'], this.maxBody);
      } catch (e) {
        return done(e.tooLarge ? GRPC_RESOURCE_EXHAUSTED : GRPC_INVALID_ARGUMENT, e.message);
      }
      return (async () => {
        for (const m of msgs) await this.onTraces(m);
      })().then(() => done(GRPC_OK, null, grpcFrame(Buffer.alloc(0))),  // empty ExportTraceServiceResponse
        (e) => done(e.refused ? GRPC_UNAVAILABLE : isBadRequest(e) ? GRPC_INVALID_ARGUMENT : GRPC_INTERNAL, e.message));
    }, (e) => done(GRPC_INVALID_ARGUMENT, e.message));
  }
}

function listen(server, port, host) {
  return new Promise((resolve, reject) => {
    server.once('error', reject);
    server.listen(port, host, () => { server.removeListener('error', reject); resolve(); });
  });
}

function readBody(stream, max) {
  return new Promise((resolve, reject) => {
    const chunks = [];
    let n = 0;
    stream.on('data', (c) => {
      n += c.length;
      if (n > max) {
        const e = new Error('request body too large');
        e.tooLarge = true;
        stream.destroy();
        reject(e);
        return;
      }
      chunks.push(c);
    });
    stream.on('end', () => resolve(Buffer.concat(chunks, n)));
    stream.on('error', reject);
  });
}

/** gRPC length-prefixed messages: [compressed u8][length u32 BE][message]. */
function grpcUnframe(buf, encoding, max = Infinity) {
  const out = [];
  let p = 0;
  while (p < buf.length) {
    if (p + 5 > buf.length) throw new Error('truncated gRPC frame');
    const compressed = buf[p], len = buf.readUInt32BE(p + 1);
    if (p + 5 + len > buf.length) throw new Error('truncated gRPC message');
    const msg = buf.subarray(p + 5, p + 5 + len);
    out.push(compressed ? inflate(msg, encoding || 'gzip', max) : msg);
    p += 5 + len;
  }
  return out;
}

function grpcFrame(msg) {
  const b = Buffer.alloc(5 + msg.length);
  b[0] = 0;
  b.writeUInt32BE(msg.length, 1);
  msg.copy(b, 5);
  return b;
}

/** otlphttp exporter: POST ExportMetricsServiceRequest bytes to {endpoint}/v1/metrics. */
class OtlpHttpExporter {
  constructor({ endpoint, timeoutMs = 10000, headers = {} }) {
    this.url = new URL(endpoint.replace(/\/+$/, '') + '/v1/metrics');
    this.timeoutMs = timeoutMs;
    this.headers = headers;
    this.sent = 0;
    this.failed = 0;
  }

  export(bytes) {
    return new Promise((resolve, reject) => {
      const req = http.request(this.url, { method: 'POST', timeout: this.timeoutMs,
        headers: Object.assign({ 'Content-Type': 'application/x-protobuf', 'Content-Length': bytes.length },
          this.headers) }, (res) => {
        res.resume();
        res.on('end', () => {
          if (res.statusCode >= 200 && res.statusCode < 300) { this.sent += 1; resolve(res.statusCode); } else {
            this.failed += 1;
            reject(new Error(`otlphttp export: HTTP ${res.statusCode}`));
          }
        });
      });
      req.on('timeout', () => req.destroy(new Error('otlphttp export: timeout')));
      req.on('error', (e) => { this.failed += 1; reject(e); });
      req.end(bytes);
    });
  }
}

module.exports = { OtlpReceiver, OtlpHttpExporter, MemoryLimiter, RefusedError, grpcFrame, grpcUnframe,
  TRACE_EXPORT_PATH };
