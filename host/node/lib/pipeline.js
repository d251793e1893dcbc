'use strict';
/**
 * The demo collector's traces -> spanmetrics -> metrics path as one object
 * (/root/reference/src/otel-collector/otelcol-config.yml:118-127):
 *
 *   traces:  receivers [otlp] -> processors [memory_limiter, transform, batch]
 *            -> exporters [spanmetrics]
 *   metrics: receivers [spanmetrics] -> exporters [otlphttp/prometheus]
 *
 * `batch` is the connector's column buffer (spans are handed to the GPU in
 * batches of `spanmetrics.batch_size`).  The other exporters of the demo's
 * traces pipeline (Jaeger, debug) are outside this path.
 */
const fs = require('fs');
const otlp = require('./otlp');
const collectorConfig = require('./collector_config');
const { SpanMetricsConnector } = require('./connector');
const { OtlpReceiver, OtlpHttpExporter, MemoryLimiter } = require('./receiver');
const { DEMO_SPAN_NAME_RULES } = require('./transform');

class TracesToMetricsPipeline {
  /**
   * @param opts.spanmetrics  connector config (YAML field names)
   * @param opts.transform    span-name rules (default: the demo collector's two rules,
   *                          otelcol-config.yml:106-113; [] = none; fromCollectorConfig
   *                          derives them from the collector config's transform processors)
   * @param opts.memoryLimiter MemoryLimiter options (default: the demo's 80% / 25%), or false
   * @param opts.receiver     OtlpReceiver options ({httpPort, grpcPort, host}), or false
   * @param opts.exporter     OtlpHttpExporter options ({endpoint}), or false
   * @param opts.addon, opts.clock  passed to the connector
   * @param opts.queue        requests received within one event-loop turn are handed to
   *                          the connector together (consumeTracesBatch: decoded on the
   *                          native columnizer's threads); default on, false = one at a time
   */
  constructor(opts = {}) {
    this.rules = opts.transform !== undefined ? opts.transform : DEMO_SPAN_NAME_RULES;
    this.limiter = opts.memoryLimiter === false ? null
      : new MemoryLimiter(Object.assign({ limit_percentage: 80, spike_limit_percentage: 25 }, opts.memoryLimiter));
    this.exporter = opts.exporter ? new OtlpHttpExporter(opts.exporter) : null;
    this.connector = new SpanMetricsConnector(opts.spanmetrics || {}, { addon: opts.addon, clock: opts.clock,
      rules: this.rules, native: opts.native, metricsConsumer: (req) => this._export(req) });
    this.receiver = opts.receiver === false ? null
      : new OtlpReceiver(Object.assign({}, opts.receiver, {
        onTraces: (b) => (this.queueOn ? this.consumeTracesQueued(b) : this.consumeTraces(b)) }));
    this.queueOn = opts.queue !== false;
    this.queueMax = 256;  // requests per consumeTracesBatch call
    this.pending = [];
    this.exportErrors = 0;
    this.lastExport = null;
  }

  async start() {
    if (this.receiver) await this.receiver.start();
    this.connector.start();
    return this;
  }

  /** memory_limiter -> (decode, transform, columnise: inside the connector) -> spanmetrics. */
  consumeTraces(bytes) {
    if (this.limiter) this.limiter.check();
    this.connector.consumeTraces(bytes);
  }

  /**
   * Queued ConsumeTraces: resolves (or rejects with what consumeTraces would
   * have thrown) once the request has been aggregated.  The memory limiter
   * refuses at enqueue time, as the synchronous path does.
   */
  consumeTracesQueued(bytes) {
    if (this.limiter) this.limiter.check();
    return new Promise((resolve, reject) => {
      this.pending.push({ bytes, resolve, reject });
      if (this.pending.length === 1) setImmediate(() => this._drainQueue());
      else if (this.pending.length >= this.queueMax) this._drainQueue();
    });
  }

  _drainQueue() {
    while (this.pending.length) {
      const batch = this.pending.splice(0, this.queueMax);
      let errs;
      try {
        errs = this.connector.consumeTracesBatch(batch.map((p) => p.bytes));
      } catch (e) {
        errs = batch.map(() => e);
      }
      batch.forEach((p, i) => (errs[i] ? p.reject(errs[i]) : p.resolve()));
    }
  }

  _export(req) {
    const bytes = otlp.encodeMetrics(req);
    this.lastExport = bytes;
    if (!this.exporter) return Promise.resolve(bytes);
    return this.exporter.export(bytes).then(() => bytes, (e) => {
      this.exportErrors += 1;
      throw e;
    });
  }

  /** One export now (what the connector's ticker does every metrics_flush_interval). */
  flush() { return this._export(this.connector.exportMetrics()); }

  async shutdown() {
    if (this.receiver) await this.receiver.close();
    this.connector.shutdown();
  }
}

/**
 * The pipeline a collector config describes: the traces pipeline that exports
 * to `spanmetrics` (its transform processors' span-name rules, in pipeline
 * order, and its memory limiter) and the connector's config block.  `configs`
 * are YAML texts, or file paths when `opts.files` is set, merged like repeated
 * `--config` flags (docker-compose.yml:756 passes otelcol-config.yml and
 * otelcol-config-extras.yml).  `opts` overrides / adds the host's own options
 * (addon, receiver, exporter, clock, and spanmetrics fields such as
 * key_capacity).
 */
TracesToMetricsPipeline.fromCollectorConfig = function fromCollectorConfig(configs, opts = {}) {
  const texts = [].concat(configs).map((c) => (opts.files ? fs.readFileSync(c, 'utf8') : c));
  const cfg = collectorConfig.loadCollectorConfig(texts, opts.env || process.env);
  const derived = collectorConfig.pipelineOptions(cfg, opts.connectorName || 'spanmetrics');
  const o = Object.assign({}, opts, {
    spanmetrics: Object.assign({}, derived.spanmetrics, opts.spanmetrics),
    transform: derived.transform,
    memoryLimiter: opts.memoryLimiter !== undefined ? opts.memoryLimiter : derived.memoryLimiter,
  });
  const p = new TracesToMetricsPipeline(o);
  p.collectorConfig = cfg;
  p.wiring = derived.wiring;
  return p;
};

module.exports = { TracesToMetricsPipeline };
