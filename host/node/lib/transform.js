'use strict';
/**
 * The demo collector's `transform` processor rules for span names, applied by
 * the host before keying (SURVEY.md a3, A12;
 * /root/reference/src/otel-collector/otelcol-config.yml:106-113):
 *
 *   replace_pattern(name, "\\?.*", "")          -- Go regexp ReplaceAllString
 *   replace_match(name, "GET /api/products/*", "GET /api/products/{productId}")
 *                                               -- whole-value glob match
 *
 * error_mode: ignore -- a rule that fails leaves the name unchanged.
 */

/** OTTL replace_match glob (gobwas/glob, no separators): `*` any run, `?` one char. */
function globToRegExp(glob) {
  let re = '^';
  for (const ch of glob) {
    if (ch === '*') re += '[\\s\\S]*';
    else if (ch === '?') re += '[\\s\\S]';
    else re += ch.replace(/[.*+?^${}()|[\]\\/]/g, '\\$&');
  }
  return new RegExp(re + '$', 'u');  // `?` matches one code point, as in Go
}

/**
 * replace_pattern(name, pattern, replacement): JS RegExp semantics, except
 * the demo's `\?.*`, which is given Go's meaning (`.` stops only at '\n').
 * Rules with a `.native` descriptor also run in the native columnizer.
 */
function replacePattern(pattern, replacement) {
  const goStrip = pattern === '\\?.*' && replacement === '';
  const re = goStrip ? /\?[^\n]*/g : new RegExp(pattern, 'g');
  const rule = (name) => name.replace(re, replacement);
  if (goStrip) rule.native = { kind: 'strip_query' };
  return rule;
}

/** replace_match(name, glob, replacement): whole-value glob with `*` and `?`. */
function replaceMatch(glob, replacement) {
  const re = globToRegExp(glob);
  const rule = (name) => (re.test(name) ? replacement : name);
  if (!/[[\]{}\\]/.test(glob)) rule.native = { kind: 'glob', pattern: glob, replacement };
  return rule;
}

/** The two statements of otelcol-config.yml:111-113, in order. */
const DEMO_SPAN_NAME_RULES = [
  replacePattern('\\?.*', ''),
  replaceMatch('GET /api/products/*', 'GET /api/products/{productId}'),
];

function applyRules(name, rules = DEMO_SPAN_NAME_RULES) {
  for (const r of rules) {
    try { name = r(name); } catch (e) { /* error_mode: ignore */ }
  }
  return name;
}

module.exports = { globToRegExp, replacePattern, replaceMatch, DEMO_SPAN_NAME_RULES, applyRules };
