'use strict';
/**
 * The demo collector's own configuration file as this host's configuration:
 * `otelcol-contrib --config=otelcol-config.yml --config=otelcol-config-extras.yml`
 * (/root/reference/docker-compose.yml:756) read into the pieces of the
 * traces -> spanmetrics -> metrics path:
 *
 *   connectors.spanmetrics                 -> SpanMetricsConnector config
 *                                             (otelcol-config.yml:115-116: empty
 *                                             body = createDefaultConfig)
 *   processors.transform.trace_statements  -> span-name rules (transform.js)
 *                                             (otelcol-config.yml:106-113)
 *   processors.memory_limiter              -> MemoryLimiter options (:102-105)
 *   service.pipelines                      -> the wiring check (:118-127)
 *
 * The YAML reader covers what collector configs use: block mappings and
 * sequences, plain / single- / double-quoted scalars, flow sequences and
 * mappings, comments, `${env:NAME}` substitution (the collector's default
 * expansion), and the multi-file deep merge of repeated --config flags.
 */
const { replacePattern, replaceMatch } = require('./transform');

// ------------------------------------------------------------------ YAML

class YamlError extends Error {}

function stripComment(line) {
  let q = null;
  for (let i = 0; i < line.length; i++) {
    const c = line[i];
    if (q) {
      if (q === '"' && c === '\\') i++;
      else if (c === q) q = null;
    } else if (c === '"' || c === "'") {
      q = c;
    } else if (c === '#' && (i === 0 || line[i - 1] === ' ' || line[i - 1] === '\t')) {
      return line.slice(0, i);
    }
  }
  return line;
}

function unescapeDouble(s, lineNo) {
  const map = { n: '\n', t: '\t', r: '\r', '"': '"', '\\': '\\', '/': '/', '0': '\0', b: '\b', f: '\f', ' ': ' ' };
  let out = '';
  for (let i = 0; i < s.length; i++) {
    if (s[i] !== '\\') { out += s[i]; continue; }
    const c = s[++i];
    if (c in map) out += map[c];
    else if (c === 'x' || c === 'u' || c === 'U') {
      const n = c === 'x' ? 2 : c === 'u' ? 4 : 8;
      out += String.fromCodePoint(parseInt(s.slice(i + 1, i + 1 + n), 16));
      i += n;
    } else throw new YamlError(`line ${lineNo}: bad escape \\${c}`);
  }
  return out;
}

function plainScalar(s) {
  if (s === '' || s === '~' || s === 'null' || s === 'Null' || s === 'NULL') return null;
  if (/^(true|True|TRUE)$/.test(s)) return true;
  if (/^(false|False|FALSE)$/.test(s)) return false;
  if (/^[-+]?[0-9]+$/.test(s)) return Number(s);
  if (/^0x[0-9a-fA-F]+$/.test(s)) return parseInt(s, 16);
  if (/^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$/.test(s)) return Number(s);
  return s;
}

/** One flow or quoted or plain scalar value (the text after `key:` or `- `). */
function parseValue(text, lineNo) {
  const t = text.trim();
  if (t[0] === '"') {
    if (t[t.length - 1] !== '"' || t.length < 2) throw new YamlError(`line ${lineNo}: unterminated string`);
    return unescapeDouble(t.slice(1, -1), lineNo);
  }
  if (t[0] === "'") {
    if (t[t.length - 1] !== "'" || t.length < 2) throw new YamlError(`line ${lineNo}: unterminated string`);
    return t.slice(1, -1).replace(/''/g, "'");
  }
  if (t[0] === '[' || t[0] === '{') {
    const p = { s: t, i: 0 };
    const v = parseFlow(p, lineNo);
    if (p.s.slice(p.i).trim() !== '') throw new YamlError(`line ${lineNo}: trailing text after flow value`);
    return v;
  }
  return plainScalar(t);
}

function parseFlow(p, lineNo) {
  const ws = () => { while (p.i < p.s.length && /\s/.test(p.s[p.i])) p.i++; };
  const item = () => {
    ws();
    const c = p.s[p.i];
    if (c === '[' || c === '{') return parseFlow(p, lineNo);
    if (c === '"' || c === "'") {
      let j = p.i + 1;
      while (j < p.s.length && p.s[j] !== c) j += p.s[j] === '\\' && c === '"' ? 2 : 1;
      const v = parseValue(p.s.slice(p.i, j + 1), lineNo);
      p.i = j + 1;
      return v;
    }
    let j = p.i;
    while (j < p.s.length && !',]}:'.includes(p.s[j])) j++;
    const v = plainScalar(p.s.slice(p.i, j).trim());
    p.i = j;
    return v;
  };
  const open = p.s[p.i++];
  const close = open === '[' ? ']' : '}';
  const out = open === '[' ? [] : {};
  ws();
  if (p.s[p.i] === close) { p.i++; return out; }
  for (;;) {
    if (open === '[') out.push(item());
    else {
      const k = item();
      ws();
      if (p.s[p.i] !== ':') throw new YamlError(`line ${lineNo}: expected ':' in flow mapping`);
      p.i++;
      out[String(k)] = item();
    }
    ws();
    const c = p.s[p.i++];
    if (c === close) return out;
    if (c !== ',') throw new YamlError(`line ${lineNo}: expected ',' or '${close}' in flow value`);
  }
}

function keyValue(text, lineNo) {
  // `key: value` / `key:`; the key may be quoted
  let k, rest;
  if (text[0] === '"' || text[0] === "'") {
    const q = text[0];
    let j = 1;
    while (j < text.length && text[j] !== q) j += text[j] === '\\' && q === '"' ? 2 : 1;
    k = parseValue(text.slice(0, j + 1), lineNo);
    rest = text.slice(j + 1);
    if (!/^\s*:(\s|$)/.test(rest)) return null;
    rest = rest.replace(/^\s*:/, '');
  } else {
    const m = /^([^\s"'#][^:]*?)\s*:(\s+|$)(.*)$/.exec(text);
    if (!m) return null;
    k = m[1];
    rest = m[3];
  }
  return { key: String(k), rest: rest.trim() };
}

/** Parse YAML text (the collector-config subset) into plain JS values. */
function parseYaml(text) {
  const lines = [];
  text.split(/\r?\n/).forEach((raw, i) => {
    if (raw.includes('\t') && /^\s*\t/.test(raw)) throw new YamlError(`line ${i + 1}: tab indentation`);
    const body = stripComment(raw).replace(/\s+$/, '');
    if (body.trim() === '' || body.trim() === '---') return;
    const indent = body.length - body.trimStart().length;
    lines.push({ indent, text: body.trimStart(), no: i + 1 });
  });
  let pos = 0;
  const isSeq = (l) => l.text === '-' || l.text.startsWith('- ');

  function block(indent) {
    if (pos >= lines.length || lines[pos].indent < indent) return null;
    return isSeq(lines[pos]) ? seq(lines[pos].indent) : map(lines[pos].indent);
  }
  function seq(indent) {
    const out = [];
    while (pos < lines.length && lines[pos].indent === indent && isSeq(lines[pos])) {
      const l = lines[pos];
      const rest = l.text === '-' ? '' : l.text.slice(2);
      const lead = l.text === '-' ? 1 : 2 + (rest.length - rest.trimStart().length);
      const r = rest.trim();
      if (r === '') {
        pos++;
        out.push(pos < lines.length && lines[pos].indent > indent ? block(indent + 1) : null);
      } else if (keyValue(r, l.no) && r[0] !== '[' && r[0] !== '{') {
        // a mapping that starts on the item's line: re-read this line as the
        // mapping's first key at the column where it starts
        lines[pos] = { indent: indent + lead, text: r, no: l.no };
        out.push(map(indent + lead));
      } else {
        pos++;
        out.push(parseValue(r, l.no));
      }
    }
    return out;
  }
  function map(indent) {
    const out = {};
    while (pos < lines.length && lines[pos].indent === indent && !isSeq(lines[pos])) {
      const l = lines[pos];
      const kv = keyValue(l.text, l.no);
      if (!kv) throw new YamlError(`line ${l.no}: expected 'key: value'`);
      pos++;
      if (kv.rest !== '') {
        out[kv.key] = parseValue(kv.rest, l.no);
      } else if (pos < lines.length && (lines[pos].indent > indent ||
                 (lines[pos].indent === indent && isSeq(lines[pos])))) {
        out[kv.key] = lines[pos].indent > indent ? block(indent + 1) : seq(indent);
      } else {
        out[kv.key] = null;
      }
    }
    if (pos < lines.length && lines[pos].indent > indent)
      throw new YamlError(`line ${lines[pos].no}: unexpected indentation`);
    return out;
  }
  const v = lines.length ? block(0) : null;
  if (pos !== lines.length) throw new YamlError(`line ${lines[pos].no}: unexpected content`);
  return v;
}

/** The collector's ${env:NAME} / ${NAME} expansion over every string. */
function expandEnv(v, env) {
  if (typeof v === 'string') {
    return v.replace(/\$\{(?:env:)?([A-Za-z_][A-Za-z0-9_]*)(?::-([^}]*))?\}/g,
      (_, name, dflt) => (env[name] !== undefined ? env[name] : dflt !== undefined ? dflt : ''));
  }
  if (Array.isArray(v)) return v.map((x) => expandEnv(x, env));
  if (v && typeof v === 'object') {
    const o = {};
    for (const k of Object.keys(v)) o[k] = expandEnv(v[k], env);
    return o;
  }
  return v;
}

/** Repeated --config files: later maps merge into earlier ones, other values replace. */
function deepMerge(a, b) {
  if (b === undefined) return a;
  if (a && b && typeof a === 'object' && typeof b === 'object' && !Array.isArray(a) && !Array.isArray(b)) {
    const o = Object.assign({}, a);
    for (const k of Object.keys(b)) o[k] = k in a ? deepMerge(a[k], b[k]) : b[k];
    return o;
  }
  return b;
}

function loadCollectorConfig(texts, env = process.env) {
  let cfg = {};
  for (const t of [].concat(texts)) cfg = deepMerge(cfg, parseYaml(t) || {});
  return expandEnv(cfg, env);
}

// ------------------------------------------------------------------ OTTL

class ConfigError extends Error {}

/** OTTL string literal: double-quoted, backslash escapes. */
function ottlArgs(argText, stmt) {
  const args = [];
  let i = 0;
  const s = argText;
  while (i < s.length) {
    while (i < s.length && /\s/.test(s[i])) i++;
    if (s[i] === '"') {
      let j = i + 1, v = '';
      while (j < s.length && s[j] !== '"') {
        if (s[j] === '\\') {
          const c = s[j + 1];
          v += c === 'n' ? '\n' : c === 't' ? '\t' : c === 'r' ? '\r' : c;
          j += 2;
        } else v += s[j++];
      }
      if (j >= s.length) throw new ConfigError(`unterminated string in OTTL statement: ${stmt}`);
      args.push({ str: v });
      i = j + 1;
    } else {
      let j = i;
      while (j < s.length && s[j] !== ',') j++;
      args.push({ path: s.slice(i, j).trim() });
      i = j;
    }
    while (i < s.length && /\s/.test(s[i])) i++;
    if (i < s.length) {
      if (s[i] !== ',') throw new ConfigError(`cannot parse OTTL arguments: ${stmt}`);
      i++;
    }
  }
  return args;
}

/**
 * One span-context OTTL statement on the span name -> a rule function
 * (transform.js).  Supported: replace_pattern(name, re, repl) and
 * replace_match(name, glob, repl), the two editors the demo uses.
 */
function ottlRule(stmt) {
  const m = /^\s*([a-z_]+)\s*\((.*)\)\s*(?:where\s+.*)?$/s.exec(stmt);
  if (!m) throw new ConfigError(`cannot parse OTTL statement: ${stmt}`);
  if (/\)\s*where\s/.test(stmt)) throw new ConfigError(`OTTL where-clauses are not supported: ${stmt}`);
  const args = ottlArgs(m[2], stmt);
  const target = args[0] && args[0].path;
  if (target !== 'name') throw new ConfigError(`only statements on the span name are supported: ${stmt}`);
  if (args.length !== 3 || !('str' in args[1]) || !('str' in args[2]))
    throw new ConfigError(`expected ${m[1]}(name, "<pattern>", "<replacement>"): ${stmt}`);
  if (m[1] === 'replace_pattern') return replacePattern(args[1].str, args[2].str);
  if (m[1] === 'replace_match') return replaceMatch(args[1].str, args[2].str);
  throw new ConfigError(`unsupported OTTL editor ${m[1]}: ${stmt}`);
}

/** processors.<name>.trace_statements (span context) -> ordered rules. */
function transformRules(cfg, name = 'transform') {
  const p = ((cfg && cfg.processors) || {})[name];
  if (!p) return [];
  const groups = p.trace_statements || [];
  const rules = [];
  for (const g of groups) {
    if (typeof g === 'string') { rules.push(ottlRule(g)); continue; }  // flat form: span context
    const ctx = g.context || 'span';
    if (ctx !== 'span') throw new ConfigError(`trace_statements context ${ctx} is not supported`);
    if (g.conditions) throw new ConfigError('trace_statements conditions are not supported');
    for (const st of g.statements || []) rules.push(ottlRule(st));
  }
  rules.errorMode = p.error_mode || 'propagate';
  return rules;
}

/** connectors.<name> (null = empty body = createDefaultConfig). */
function spanmetricsConfig(cfg, name = 'spanmetrics') {
  const c = (cfg && cfg.connectors) || {};
  if (!(name in c)) throw new ConfigError(`connectors.${name} is not declared`);
  return c[name] || {};
}

function memoryLimiterConfig(cfg, name = 'memory_limiter') {
  const p = ((cfg && cfg.processors) || {})[name];
  return p === undefined ? null : p || {};
}

/**
 * The wiring the drop-in needs: spanmetrics is an exporter of a traces
 * pipeline and a receiver of a metrics pipeline; returns that traces
 * pipeline's processors (in order) and the metrics pipeline's exporters.
 */
function spanmetricsWiring(cfg, name = 'spanmetrics') {
  const pipes = ((cfg && cfg.service) || {}).pipelines || {};
  let traces = null, metrics = null;
  for (const [pname, p] of Object.entries(pipes)) {
    const kind = pname.split('/')[0];
    if (kind === 'traces' && (p.exporters || []).includes(name)) traces = { name: pname, processors: p.processors || [] };
    if (kind === 'metrics' && (p.receivers || []).includes(name)) metrics = { name: pname, exporters: p.exporters || [] };
  }
  if (!traces) throw new ConfigError(`no traces pipeline exports to ${name}`);
  if (!metrics) throw new ConfigError(`no metrics pipeline receives from ${name}`);
  return { traces, metrics };
}

/**
 * Options for TracesToMetricsPipeline from a collector config: the
 * connector's config, the span-name rules of the transform processors the
 * traces pipeline runs (in pipeline order), the memory limiter.
 */
function pipelineOptions(cfg, name = 'spanmetrics') {
  const wiring = spanmetricsWiring(cfg, name);
  const rules = [];
  let limiter = false;
  for (const proc of wiring.traces.processors) {
    const kind = proc.split('/')[0];
    if (kind === 'transform') {
      const r = transformRules(cfg, proc);
      rules.push(...r);
      rules.errorMode = r.errorMode;
    }
    else if (kind === 'memory_limiter') limiter = memoryLimiterConfig(cfg, proc);
  }
  return { spanmetrics: spanmetricsConfig(cfg, name), transform: rules, memoryLimiter: limiter, wiring };
}

module.exports = { parseYaml, loadCollectorConfig, expandEnv, deepMerge, ottlRule, transformRules,
  spanmetricsConfig, memoryLimiterConfig, spanmetricsWiring, pipelineOptions, YamlError, ConfigError };
