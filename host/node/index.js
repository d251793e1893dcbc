'use strict';
/** Public surface of the Node host (see INTEGRATION.md section 3). */
const addon = require('./lib/addon');
const otlp = require('./lib/otlp');
const keys = require('./lib/keys');
const transform = require('./lib/transform');
const { SpanMetricsConnector, normalizeConfig } = require('./lib/connector');
const { OtlpReceiver, OtlpHttpExporter, MemoryLimiter } = require('./lib/receiver');
const { TracesToMetricsPipeline } = require('./lib/pipeline');

module.exports = { loadAddon: addon.load, otlp, keys, transform, SpanMetricsConnector, normalizeConfig,
  OtlpReceiver, OtlpHttpExporter, MemoryLimiter, TracesToMetricsPipeline };
