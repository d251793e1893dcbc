'use strict';
/**
 * Test server for tests/test_node_host.py: an OtlpReceiver on ephemeral
 * ports that decodes every request.  Prints {"http": port, "grpc": port} on
 * start; when stdin closes, prints {"requests": n, "spans": m, "names": [...]}
 * and exits.
 */
const path = require('path');
const otlp = require(path.join(__dirname, '..', 'lib', 'otlp'));
const { OtlpReceiver } = require(path.join(__dirname, '..', 'lib', 'receiver'));

let requests = 0, spans = 0;
const names = [];
const rx = new OtlpReceiver({ httpPort: 0, grpcPort: 0, onTraces: (b) => {
  requests += 1;
  for (const rs of otlp.decodeTraces(b).resourceSpans) {
    for (const ss of rs.scopeSpans) for (const s of ss.spans) { spans += 1; names.push(s.name); }
  }
} });
rx.start().then(() => {
  process.stdout.write(JSON.stringify({ http: rx.httpPort, grpc: rx.grpcPort }) + '\n');
  process.stdin.resume();
  process.stdin.on('end', async () => {
    await rx.close();
    process.stdout.write(JSON.stringify({ requests, spans, names }) + '\n');
    process.exit(0);
  });
});
