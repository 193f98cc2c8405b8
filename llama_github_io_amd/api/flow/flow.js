// Flow: the notebook web UI of the REST server (reference: h2o-web, which serves the h2o-flow notebook at
// /flow/index.html; the notebooks it ships are h2o-docs/src/product/flow/packs/**/*.flow).
//
// A Flow notebook is a list of cells ({type: "cs" | "md" | "h1".."h6" | "raw", input}); a "cs" cell holds one
// routine call in Flow's CoffeeScript syntax:
//   getFrames
//   importFiles ["data.csv"]
//   parseFiles                                  <- an implicit object over indented lines
//     paths: ["data.csv"]
//     destination_frame: "data.hex"
//   buildModel 'gbm', {"training_frame": "data.hex", "response_column": "y", "ntrees": "50"}
//   predict model: "m", frame: "f"
//   inspect getModel "m"                         <- nested implicit calls
//   grid inspect 'summary', getGrid "g", sort_by: "auc", decreasing: true
//   assist buildModel, null, training_frame: "f" <- a routine passed by name
// This file is the whole command layer: parsing a cell (parseCell: a small parser for that CoffeeScript subset —
// literals, arrays, objects, implicit objects and implicit / parenthesised calls, # comments), running it against
// the REST API (runCell, with an injected `http(method, path, body)` so the same code runs in the browser and under
// node in the tests), and rendering results as HTML (render). index.html is the page shell around it.
"use strict";

// ------------------------------------------------------------------------------------------------ parsing
// Tokens; a run of line breaks (blank and comment-only lines included) is ONE "nl" token carrying the indentation
// of the next line.
function tokenize(src) {
  const toks = [];
  let i = 0;
  const indentAt = (j) => { let k = 0; while (src[j + k] === " " || src[j + k] === "\t") k++; return k; };
  while (i < src.length) {
    const c = src[i];
    if (c === "#") { while (i < src.length && src[i] !== "\n") i++; continue; }       // comment
    if (c === "\n") {
      const ind = indentAt(i + 1);
      const last = toks[toks.length - 1];
      if (last && last.t === "nl") last.ind = ind; else toks.push({ t: "nl", ind });
      i++;
      continue;
    }
    if (/\s/.test(c)) { i++; continue; }
    if (c === '"' || c === "'") {
      let j = i + 1, s = "";
      while (j < src.length && src[j] !== c) {
        if (src[j] === "\\" && j + 1 < src.length) {
          const e = src[j + 1];
          const m = { n: "\n", t: "\t", r: "\r" }[e];
          s += m === undefined ? e : m;
          j += 2;
          continue;
        }
        s += src[j++];
      }
      if (j >= src.length) throw new Error("unterminated string");
      toks.push({ t: "str", v: s });
      i = j + 1;
      continue;
    }
    const hex = /^0[xX][0-9a-fA-F]+/.exec(src.slice(i));
    if (hex) { toks.push({ t: "num", v: parseInt(hex[0].slice(2), 16) }); i += hex[0].length; continue; }
    const num = /^(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?/.exec(src.slice(i));
    if (num) { toks.push({ t: "num", v: Number(num[0]) }); i += num[0].length; continue; }
    const id = /^[A-Za-z_$][\w$]*/.exec(src.slice(i));
    if (id) { toks.push({ t: "id", v: id[0] }); i += id[0].length; continue; }
    if ("[]{}(),:-;=+".includes(c)) { toks.push({ t: c }); i++; continue; }
    throw new Error("unexpected character " + JSON.stringify(c));
  }
  toks.push({ t: "eof" });
  return toks;
}

const LITERAL_IDS = { true: true, false: false, null: null, undefined: null, yes: true, no: false, on: true, off: false };
const KEYWORDS = { if: 1, else: 1, then: 1 };

const tokName = (x) => (x.v !== undefined ? x.v : x.t);

// AST: {lit: v} | {arr: [..]} | {obj: [[k, node], ..]} | {call: name, args: [..]} | {ref: name} | {add: [a, b]}
// statements: {expr: node} | {set: name, expr: node} | {if: node, then: [..], else: [..]}
function parseTokens(toks) {
  let p = 0;
  const peek = (k = 0) => toks[p + k];
  const next = () => toks[p++];
  const expect = (t) => { const x = next(); if (x.t !== t) throw new Error("expected " + t + " but found " + tokName(x)); return x; };
  const skipNl = () => { while (peek().t === "nl") p++; };
  const isKey = (k = 0) => (peek(k).t === "id" || peek(k).t === "str") && peek(k + 1).t === ":";
  const startsArg = (x) => ["str", "num", "[", "{", "id"].includes(x.t) && !(x.t === "id" && KEYWORDS[x.v]);

  function value() {                                     // one expression: primaries joined by +
    let v = primary();
    while (peek().t === "+") { p++; skipNl(); v = { add: [v, primary()] }; }
    return v;
  }

  function primary() {
    const x = peek();
    if (x.t === "str") { p++; return { lit: x.v }; }
    if (x.t === "num") { p++; return { lit: x.v }; }
    if (x.t === "-" && peek(1).t === "num") { p += 2; return { lit: -peek(-1).v }; }
    if (x.t === "[") return array();
    if (x.t === "{") return object();
    if (x.t === "(") { p++; skipNl(); const v = value(); skipNl(); expect(")"); return v; }
    if (x.t === "id") {
      if (Object.prototype.hasOwnProperty.call(LITERAL_IDS, x.v)) { p++; return { lit: LITERAL_IDS[x.v] }; }
      p++;
      if (peek().t === "(") {                            // name(args)
        p++;
        skipNl();
        const args = peek().t === ")" ? [] : argList(true);
        skipNl();
        expect(")");
        return { call: x.v, args };
      }
      if (startsArg(peek())) return { call: x.v, args: argList(false) };
      return { ref: x.v };
    }
    throw new Error("unexpected " + tokName(x));
  }

  function array() {
    expect("[");
    const items = [];
    for (;;) {
      while (peek().t === "nl" || peek().t === "," || peek().t === ";") p++;
      if (peek().t === "]") { p++; return { arr: items }; }
      items.push(value());
    }
  }

  function pairs(close) {                                // key: value pairs separated by commas or new lines
    const out = [];
    for (;;) {
      while (peek().t === "nl" || peek().t === ",") {
        if (!close && peek().t === "nl" && !isKeyAfterNl()) return out;
        p++;
      }
      if (close ? peek().t === close : !isKey()) return out;
      const k = next();
      if (k.t !== "id" && k.t !== "str") throw new Error("expected a key");
      expect(":");
      skipNl();
      out.push([k.v, value()]);
    }
  }

  function isKeyAfterNl() {                              // an implicit object continues on the next line
    let k = 0;
    while (peek(k).t === "nl" || peek(k).t === ",") k++;
    return (peek(k).t === "id" || peek(k).t === "str") && peek(k + 1).t === ":";
  }

  function object() {
    expect("{");
    const o = pairs("}");
    expect("}");
    return { obj: o };
  }

  // implicit-call arguments: comma separated; `key: value, ...` at the end is one object argument
  function argList(inParens) {
    const args = [];
    for (;;) {
      if (inParens) skipNl();
      if (isKey()) { args.push({ obj: pairs(inParens ? ")" : null) }); return args; }
      args.push(value());
      if (peek().t === ",") {
        p++;
        if (inParens || peek().t === "nl") skipNl();
        continue;
      }
      return args;
    }
  }

  function statement() {
    const x = peek();
    if (x.t === "id" && x.v === "if") {
      p++;
      const cond = value();
      if (peek().t === "id" && peek().v === "then") p++;
      const thenB = block();
      let elseB = [];
      const save = p;
      if (peek().t === "nl") p++;
      if (peek().t === "id" && peek().v === "else") { p++; elseB = block(); } else p = save;
      return { if: cond, then: thenB, else: elseB };
    }
    if (x.t === "id" && peek(1).t === "=") {
      p += 2;
      skipNl();
      return { set: x.v, expr: value() };
    }
    if (x.t === "id" && !LITERAL_IDS.hasOwnProperty(x.v) && peek(1).t === "nl" && (() => {
      let k = 1;
      while (peek(k).t === "nl") k++;
      return isKey(k);
    })()) {
      // `name` then an indented block of `key: value` lines (parseFiles / setupParse as Flow writes them)
      p++;
      return { expr: { call: x.v, args: [{ obj: pairs(null) }] } };
    }
    return { expr: value() };
  }

  // an indented block after `if` / `else` (or a statement on the same line)
  function block() {
    if (peek().t !== "nl") return [statement()];
    const ind = peek().ind;
    const out = [];
    while (peek().t === "nl" && peek().ind === ind && ind > 0) {
      p++;
      if (peek().t === "eof") break;
      out.push(statement());
    }
    if (!out.length) throw new Error("empty block");
    return out;
  }

  const stmts = [];
  for (;;) {
    while (peek().t === "nl" || peek().t === ";") p++;
    if (peek().t === "eof") break;
    if (peek().t === "id" && peek().v === "else") throw new Error("else without if");
    stmts.push(statement());
    if (peek().t !== "nl" && peek().t !== ";" && peek().t !== "eof")
      throw new Error("unexpected " + tokName(peek()) + " after the command");
  }
  return stmts;
}

// AST node -> plain value (nested calls stay {__call, args}; names {__ref}: a variable or a routine passed by
// name; a + b {__add})
function toValue(n) {
  if ("lit" in n) return n.lit;
  if (n.arr) return n.arr.map(toValue);
  if (n.obj) { const o = {}; for (const [k, v] of n.obj) o[k] = toValue(v); return o; }
  if (n.call) return { __call: n.call, args: n.args.map(toValue) };
  if (n.add) return { __add: n.add.map(toValue) };
  return { __ref: n.ref };
}

function toStmt(s) {
  if (s.if) return { if: toValue(s.if), then: s.then.map(toStmt), else: s.else.map(toStmt) };
  if (s.set) return { set: s.set, expr: toValue(s.expr) };
  return { expr: toValue(s.expr) };
}

// a cell -> {name, args} when it is one routine call, {script: [statements]} otherwise (assignments, if / else)
function parseCell(text) {
  const src = String(text || "").replace(/\r\n/g, "\n");
  if (!src.trim()) return null;
  let st;
  try {
    st = parseTokens(tokenize(src));
  } catch (e) {
    const name = (/^\s*([A-Za-z_]\w*)/.exec(src) || [])[1] || "cell";
    throw new Error("cannot parse the arguments of " + name + ": " + e.message);
  }
  if (!st.length) return null;
  if (st.length === 1 && st[0].expr && (st[0].expr.call || st[0].expr.ref)) {
    const e = st[0].expr;
    return { name: e.call || e.ref, args: (e.args || []).map(toValue) };
  }
  return { script: st.map(toStmt) };
}

// the pre-parser name kept for callers of the JSON-subset converter
function toJSON(src) { return JSON.stringify(toValue(parseTokens(tokenize("x " + src))[0].expr.args[0] || { lit: null })); }

// ------------------------------------------------------------------------------------------------ commands
const enc = encodeURIComponent;
const keyName = (k) => (k && typeof k === "object" ? k.name : k);
const isCall = (v) => v && typeof v === "object" && typeof v.__call === "string";

async function evalArg(http, v, opts) {
  if (isCall(v)) return runCommand(http, v.__call, v.args, opts);
  if (v && typeof v === "object" && typeof v.__ref === "string") {
    const sc = (opts && opts.scope) || {};
    if (Object.prototype.hasOwnProperty.call(sc, v.__ref)) return sc[v.__ref];
    if (COMMANDS[v.__ref]) return v;                      // a routine passed by name (assist buildModel)
    throw new Error(v.__ref + " is not defined");
  }
  if (v && typeof v === "object" && Array.isArray(v.__add)) {
    const [a, b] = [await evalArg(http, v.__add[0], opts), await evalArg(http, v.__add[1], opts)];
    return a + b;
  }
  if (Array.isArray(v)) { const o = []; for (const x of v) o.push(await evalArg(http, x, opts)); return o; }
  if (v && typeof v === "object" && !v.__ref && !v.kind) {
    const o = {};
    for (const k of Object.keys(v)) o[k] = await evalArg(http, v[k], opts);
    return o;
  }
  return v;
}

async function waitJob(http, job, opts) {
  const key = keyName(job.key);
  if (!key || job.status === "DONE") return job;
  const poll = (opts && opts.pollMs) || 200;
  for (let i = 0; ; i++) {
    const r = await http("GET", "/3/Jobs/" + enc(key));
    const j = r.jobs[0];
    if (j.status === "DONE") return j;
    if (j.status === "FAILED" || j.status === "CANCELLED")
      throw new Error("job " + key + " " + j.status.toLowerCase() + ": " + (j.exception || j.progress_msg || ""));
    if (opts && opts.maxPolls && i >= opts.maxPolls) throw new Error("job " + key + " still running");
    await new Promise((res) => setTimeout(res, poll));
  }
}

async function frameSummary(h, f) { return (await h("GET", "/3/Frames/" + enc(f) + "/summary")).frames[0]; }

async function columnIndex(h, f, col) {
  const s = await frameSummary(h, f);
  const i = (s.columns || []).findIndex((c) => c.label === col);
  if (i < 0) throw new Error("no column " + col + " in " + f);
  return [i, s];
}

// Rapids string literal
const rq = (s) => '"' + String(s).replace(/\\/g, "\\\\").replace(/"/g, '\\"') + '"';

// parameter values as Flow's forms send them (numbers as strings, "" for unset) -> the REST form
function cleanParams(o) {
  const out = {};
  for (const [k, v] of Object.entries(o || {})) {
    if (v === "" || v === null || v === undefined) continue;
    if (Array.isArray(v) && v.length === 0 && !["ignored_columns"].includes(k)) continue;
    out[k] = v;
  }
  return out;
}

const COMMANDS = {
  help: { doc: "list the commands", run: async () => ({ kind: "help", data: Object.keys(COMMANDS).sort().map(
    (k) => ({ command: k, description: COMMANDS[k].doc })) }) },
  assist: { doc: "assist [routine, args...]: the routines menu (Flow's Assist Me), or the form a routine needs",
    run: async (h, args) => {
      const [fn, ...rest] = args;
      if (fn && fn.__ref) {
        const d = { routine: fn.__ref, doc: (COMMANDS[fn.__ref] || {}).doc || "", args: rest.filter((a) => a !== null) };
        if (fn.__ref === "buildModel")
          d.algos = Object.keys((await h("GET", "/3/ModelBuilders")).model_builders).sort();
        return { kind: "assist", data: d };
      }
      return COMMANDS.help.run(h, []);
    } },
  getCloud: { doc: "cluster status", run: async (h) => ({ kind: "cloud", data: await h("GET", "/3/Cloud") }) },
  getTimeline: { doc: "recent REST events", run: async (h) => ({ kind: "json", data: await h("GET", "/3/Timeline") }) },
  getFrames: { doc: "list frames", run: async (h) => ({ kind: "frames", data: (await h("GET", "/3/Frames")).frames }) },
  getFrame: { doc: 'getFrame "frame": the frame with its column summaries',
    run: async (h, [f]) => ({ kind: "frameSummary", data: await frameSummary(h, keyName(f)) }) },
  getFrameSummary: { doc: 'getFrameSummary "frame": column summaries',
    run: async (h, [f]) => ({ kind: "frameSummary", data: await frameSummary(h, keyName(f)) }) },
  getColumnSummary: { doc: 'getColumnSummary "frame", "column"',
    run: async (h, [f, c]) => {
      const r = (await h("GET", "/3/Frames/" + enc(keyName(f)) + "/columns/" + enc(c) + "/summary")).frames[0];
      return { kind: "frameSummary", data: r };
    } },
  getFrameData: { doc: 'getFrameData "frame": the first rows',
    run: async (h, [f, n]) => ({ kind: "frameData",
      data: (await h("GET", "/3/Frames/" + enc(keyName(f)) + "?row_count=" + (n || 10))).frames[0] }) },
  deleteFrame: { doc: 'deleteFrame "frame"',
    run: async (h, [f]) => { await h("DELETE", "/3/Frames/" + enc(f)); return { kind: "text", data: "deleted frame " + f }; } },
  importFiles: { doc: 'importFiles ["path", ...]: register files for parsing',
    run: async (h, [paths]) => ({ kind: "import",
      data: await h("POST", "/3/ImportFilesMulti", { paths: Array.isArray(paths) ? paths : [paths] }) }) },
  setupParse: { doc: 'setupParse paths: ["path"]: guess the parse setup',
    run: async (h, [o]) => {
      o = Object.assign({}, o);
      if (o.paths && !o.source_frames) { o.source_frames = o.paths; delete o.paths; }
      return { kind: "parseSetup", data: await h("POST", "/3/ParseSetup", o) };
    } },
  parseFiles: { doc: "parseFiles paths: [...], destination_frame: ..., column_types: [...], ...: parse into a frame",
    run: async (h, [o], opts) => {
      o = cleanParams(o);
      if (o.paths && !o.source_frames) { o.source_frames = o.paths; delete o.paths; }
      const r = await h("POST", "/3/Parse", o);
      await waitJob(h, r.job, opts);
      return { kind: "frameSummary", data: await frameSummary(h, keyName(r.destination_frame)) };
    } },
  importAndParse: { doc: 'importAndParse "path", "destination": importFiles + setupParse + parseFiles',
    run: async (h, [path, dest], opts) => {
      const imp = await h("POST", "/3/ImportFilesMulti", { paths: [path] });
      const st = await h("POST", "/3/ParseSetup", { source_frames: imp.destination_frames });
      const body = { source_frames: imp.destination_frames, destination_frame: dest || st.destination_frame,
        separator: st.separator, check_header: st.check_header, column_names: st.column_names,
        column_types: st.column_types };
      return COMMANDS.parseFiles.run(h, [body], opts);
    } },
  splitFrame: { doc: 'splitFrame "frame", [0.75], ["train", "test"], seed',
    run: async (h, [f, ratios, dests, seed]) => ({ kind: "split", data: await h("POST", "/3/SplitFrame",
      { dataset: keyName(f), ratios: ratios || [0.75], destination_frames: dests, seed: seed === undefined ? null : seed }) }) },
  createFrame: { doc: 'createFrame {dest: "f", rows: 1000, cols: 10, ...}: a random frame',
    run: async (h, [o], opts) => {
      const r = await h("POST", "/3/CreateFrame", cleanParams(o));
      if (r.job) await waitJob(h, r.job, opts);
      return { kind: "frameSummary", data: await frameSummary(h, keyName(r.key) || o.dest) };
    } },
  bindFrames: { doc: 'bindFrames "dest", ["f1", "f2"]: column-bind frames',
    run: async (h, [dest, frames]) => {
      await h("POST", "/99/Rapids", { ast: "(assign " + dest + " (cbind " + frames.map(keyName).join(" ") + "))",
        session_id: "_flow" });
      return { kind: "frameSummary", data: await frameSummary(h, dest) };
    } },
  changeColumnType: { doc: "changeColumnType frame: \"f\", column: \"c\", type: 'enum' | 'numeric' | 'string'",
    run: async (h, [o]) => {
      const f = keyName(o.frame);
      const [i] = await columnIndex(h, f, o.column);
      const t = String(o.type).toLowerCase();
      const op = t === "enum" || t === "factor" || t === "categorical" ? "as.factor" :
        t === "string" ? "as.character" : "as.numeric";
      await h("POST", "/99/Rapids", { ast: "(assign " + f + " (:= " + f + " (" + op + " (cols " + f + " [" + i + "])) [" +
        i + "] []))", session_id: "_flow" });
      return { kind: "frameSummary", data: await frameSummary(h, f) };
    } },
  imputeColumn: { doc: 'imputeColumn {frame: "f", column: "c", method: "MEAN" | "MEDIAN" | "MODE", groupByColumns: [...]}',
    run: async (h, [o]) => {
      const f = keyName(o.frame);
      const [i, s] = await columnIndex(h, f, o.column);
      const by = (o.groupByColumns || []).map((c) => (s.columns || []).findIndex((x) => x.label === c));
      if (by.some((b) => b < 0)) throw new Error("unknown group-by column");
      await h("POST", "/99/Rapids", { ast: "(h2o.impute " + f + " " + i + " " + rq(String(o.method || "mean").toLowerCase()) +
        " " + rq(String(o.combineMethod || "interpolate").toLowerCase()) + " [" + by.join(" ") + "] _ _)", session_id: "_flow" });
      return { kind: "frameSummary", data: await frameSummary(h, f) };
    } },
  exportFrame: { doc: 'exportFrame "frame", "path", overwrite: true',
    run: async (h, [f, path, o]) => {
      if (!path) return { kind: "form", data: { routine: "exportFrame", frame: keyName(f), needs: ["path"] } };
      const r = await h("POST", "/3/Frames/" + enc(keyName(f)) + "/export", { path, force: !!(o && o.overwrite) });
      return { kind: "text", data: "exported " + keyName(f) + " to " + (r.path || path) };
    } },
  getModels: { doc: "list models", run: async (h) => ({ kind: "models", data: (await h("GET", "/3/Models")).models }) },
  getModel: { doc: 'getModel "model"',
    run: async (h, [m]) => ({ kind: "model", data: (await h("GET", "/3/Models/" + enc(keyName(m)))).models[0] }) },
  deleteModel: { doc: 'deleteModel "model"',
    run: async (h, [m]) => { await h("DELETE", "/3/Models/" + enc(m)); return { kind: "text", data: "deleted model " + m }; } },
  getModelBuilders: { doc: "algorithms that can be built",
    run: async (h) => ({ kind: "builders", data: Object.keys((await h("GET", "/3/ModelBuilders")).model_builders).sort() }) },
  buildModel: { doc: "buildModel 'gbm', {training_frame: \"f\", response_column: \"y\", ...} (hyper_parameters: a grid)",
    run: async (h, [algo, params], opts) => {
      if (!algo) return COMMANDS.assist.run(h, [{ __ref: "buildModel" }]);
      params = cleanParams(params);
      if (params.hyper_parameters) {                         // Flow's grid checkbox: a grid search
        const body = Object.assign({}, params);
        const gid = body.grid_id || body.model_id;
        delete body.model_id;
        body.grid_id = gid;
        body.hyper_parameters = JSON.stringify(body.hyper_parameters);
        if (body.search_criteria) body.search_criteria = JSON.stringify(body.search_criteria);
        const r = await h("POST", "/99/Grid/" + enc(algo), body);
        await waitJob(h, r.job, opts);
        return { kind: "grid", data: await h("GET", "/99/Grids/" + enc(keyName(r.grid_id) || gid)) };
      }
      const r = await h("POST", "/3/ModelBuilders/" + enc(algo), params);
      const j = await waitJob(h, r.job, opts);
      return { kind: "model", data: (await h("GET", "/3/Models/" + enc(keyName(j.dest)))).models[0] };
    } },
  predict: { doc: 'predict model: "m", frame: "f" [, predictions_frame: "p"]',
    run: async (h, [o]) => {
      o = o || {};
      if (!o.frame) {
        const frames = (await h("GET", "/3/Frames")).frames.map((f) => keyName(f.frame_id));
        return { kind: "form", data: { routine: "predict", model: keyName(o.model), needs: ["frame"], frames } };
      }
      return { kind: "prediction", data: await h("POST", "/3/Predictions/models/" + enc(keyName(o.model)) +
        "/frames/" + enc(keyName(o.frame)), o.predictions_frame ? { predictions_frame: o.predictions_frame } : {}) };
    } },
  getPrediction: { doc: 'getPrediction model: "m", frame: "f": the metrics of a model on a frame',
    run: async (h, [o]) => ({ kind: "prediction", data: await h("GET", "/3/ModelMetrics/models/" + enc(keyName(o.model)) +
      "/frames/" + enc(keyName(o.frame))) }) },
  getGrids: { doc: "list grids", run: async (h) => ({ kind: "grids", data: (await h("GET", "/99/Grids")).grids || [] }) },
  getGrid: { doc: 'getGrid "grid", sort_by: "auc", decreasing: true',
    run: async (h, [g, o]) => {
      const q = [];
      if (o && o.sort_by) q.push("sort_by=" + enc(o.sort_by));
      if (o && o.decreasing !== undefined) q.push("decreasing=" + !!o.decreasing);
      return { kind: "grid", data: await h("GET", "/99/Grids/" + enc(keyName(g)) + (q.length ? "?" + q.join("&") : "")) };
    } },
  inspect: { doc: "inspect [table name,] result: the tables inside a result (inspect getModel \"m\")",
    run: async (h, args) => {
      const [a, b] = args;
      const name = typeof a === "string" ? a : null;
      const res = name === null ? a : b;
      if (!res || !res.kind) throw new Error("inspect needs a result, e.g. inspect getModel \"m\"");
      const tables = tablesOf(res);
      if (name === null) return { kind: "tables", data: tables };
      const t = tables.find((x) => x.name === name) || tables.find((x) => x.name.toLowerCase() === name.toLowerCase()) ||
        tables.find((x) => x.name.toLowerCase().endsWith(name.toLowerCase().replace(/^output - /, "")));
      if (!t) throw new Error("no table " + name + " (have: " + tables.map((x) => x.name).join(", ") + ")");
      return { kind: "table", data: t };
    } },
  grid: { doc: "grid <table>: show a table as a grid (grid inspect 'summary', getGrid \"g\")",
    run: async (h, [res]) => {
      if (res && res.kind === "table") return res;
      if (res && res.kind) return { kind: "tables", data: tablesOf(res) };
      throw new Error("grid needs a table, e.g. grid inspect 'summary', getGrid \"g\"");
    } },
  getJobs: { doc: "list jobs", run: async (h) => ({ kind: "jobs", data: (await h("GET", "/3/Jobs")).jobs }) },
  getJob: { doc: 'getJob "job"', run: async (h, [k]) => ({ kind: "jobs", data: (await h("GET", "/3/Jobs/" + enc(k))).jobs }) },
  cancelJob: { doc: 'cancelJob "job"',
    run: async (h, [k]) => { await h("POST", "/3/Jobs/" + enc(k) + "/cancel"); return { kind: "text", data: "cancelled " + k }; } },
  runAutoML: { doc: "runAutoML {input_spec: {...}, build_control: {...}, build_models: {...}} [, 'exec'] | {training_frame, response_column, max_models, ...}",
    run: async (h, [o], opts) => {
      if (!o) return { kind: "form", data: { routine: "runAutoML", needs: ["training_frame", "response_column"] } };
      let spec = o;
      if (!o.input_spec) {
        spec = { input_spec: { training_frame: o.training_frame, response_column: o.response_column,
            validation_frame: o.validation_frame, leaderboard_frame: o.leaderboard_frame, ignored_columns: o.ignored_columns },
          build_control: { project_name: o.project_name, nfolds: o.nfolds === undefined ? 5 : o.nfolds,
            stopping_criteria: { max_models: o.max_models, max_runtime_secs: o.max_runtime_secs, seed: o.seed } },
          build_models: { include_algos: o.include_algos, exclude_algos: o.exclude_algos } };
      }
      const r = await h("POST", "/99/AutoMLBuilder", spec);
      await waitJob(h, r.job, opts);
      const pid = r.build_control.project_name;
      return { kind: "leaderboard", data: await h("GET", "/99/Leaderboards/" + enc(pid)) };
    } },
  getLeaderboard: { doc: 'getLeaderboard "project" (or H2O\'s "project@@response")',
    run: async (h, [p]) => ({ kind: "leaderboard", data: await h("GET", "/99/Leaderboards/" + enc(p)) }) },
  runRapids: { doc: 'runRapids "(expression)": evaluate a Rapids expression',
    run: async (h, [ast]) => ({ kind: "json", data: await h("POST", "/99/Rapids", { ast, session_id: "_flow" }) }) },
  saveFlow: { doc: 'saveFlow "name": store this notebook on the server (.flow format)',
    run: async (h, [name], opts) => {
      const doc = toFlowDoc((opts && opts.cells) || []);
      await h("POST", "/3/NodePersistentStorage/notebook/" + enc(name), { value: JSON.stringify(doc) });
      return { kind: "text", data: "saved notebook " + name + " (" + doc.cells.length + " cells)" };
    } },
  loadFlow: { doc: 'loadFlow "name": the cells of a stored notebook',
    run: async (h, [name]) => {
      const r = await h("GET", "/3/NodePersistentStorage/notebook/" + enc(name));
      return { kind: "notebook", data: fromFlowDoc(JSON.parse(r.value)) };
    } },
  getFlows: { doc: "stored notebooks",
    run: async (h) => ({ kind: "json", data: (await h("GET", "/3/NodePersistentStorage/notebook")).entries }) },
};

// .flow documents: {version: "1.0.0", cells: [{type, input}]}; plain strings are "cs" cells
function toFlowDoc(cells) {
  return { version: "1.0.0", cells: cells.map((c) => (typeof c === "string" ? { type: "cs", input: c } : c)) };
}
function fromFlowDoc(doc) {
  const cells = (doc && doc.cells) || [];
  return { version: (doc && doc.version) || "1.0.0",
    cells: cells.map((c) => (typeof c === "string" ? { type: "cs", input: c } : { type: c.type || "cs", input: c.input || "" })) };
}

async function runCommand(http, name, args, opts) {
  const cmd = COMMANDS[name];
  if (!cmd) throw new Error("unknown command " + name + " (try help)");
  const vals = [];
  for (const a of args) vals.push(await evalArg(http, a, opts));
  return cmd.run(http, vals, opts || {});
}

async function runCell(http, text, opts) {
  if (text && typeof text === "object") {                 // a .flow cell
    if ((text.type || "cs") !== "cs") return { kind: "markdown", data: { type: text.type, input: text.input } };
    text = text.input;
  }
  const c = parseCell(text);
  if (!c) return { kind: "text", data: "" };
  opts = opts || {};
  if (!opts.scope) opts.scope = {};
  if (c.script) return runScript(http, c.script, opts);
  const sc = opts.scope;
  if (!COMMANDS[c.name] && Object.prototype.hasOwnProperty.call(sc, c.name) && !c.args.length)
    return { kind: "json", data: sc[c.name] };            // a cell naming a variable shows its value
  return runCommand(http, c.name, c.args, opts);
}

// statements of a script cell; variables live in opts.scope (shared by the notebook's cells, as Flow's
// CoffeeScript sandbox shares them); the result is the last statement's
async function runScript(http, stmts, opts) {
  let last = { kind: "text", data: "" };
  for (const s of stmts) {
    if (s.if !== undefined) {
      last = await runScript(http, (await evalArg(http, s.if, opts)) ? s.then : s.else, opts);
    } else if (s.set !== undefined) {
      opts.scope[s.set] = await evalArg(http, s.expr, opts);
      last = { kind: "json", data: opts.scope[s.set] };
    } else if (s.expr && typeof s.expr.__ref === "string" && COMMANDS[s.expr.__ref]) {
      last = await runCommand(http, s.expr.__ref, [], opts);
    } else {
      const v = await evalArg(http, s.expr, opts);
      last = v && v.kind ? v : { kind: "json", data: v };
    }
  }
  return last;
}

// ------------------------------------------------------------------------------------------------ tables
// TwoDimTableV3 -> {name, columns, rows}
function twoDimRows(t) {
  const n = t.rowcount || (t.data && t.data[0] ? t.data[0].length : 0);
  const rows = [];
  for (let i = 0; i < n; i++) rows.push(t.data.map((col) => col[i]));
  return { name: t.name || "", columns: (t.columns || []).map((c) => c.name), rows };
}

function tablesOf(res) {
  const d = res.data || {};
  const out = [];
  const add = (name, t) => { if (t && t.columns && t.data) out.push(Object.assign(twoDimRows(t), { name })); };
  const metrics = (prefix, mm) => {
    if (!mm) return;
    const keys = ["MSE", "RMSE", "logloss", "AUC", "pr_auc", "Gini", "mean_per_class_error", "r2", "mean_residual_deviance"];
    const rows = keys.filter((k) => mm[k] !== undefined && mm[k] !== null).map((k) => [k, mm[k]]);
    if (rows.length) out.push({ name: prefix, columns: ["metric", "value"], rows });
    if (mm.cm && mm.cm.table) add(prefix + " - Confusion Matrix", mm.cm.table);
    if (mm.thresholds_and_metric_scores) add(prefix + " - Thresholds x metric scores", mm.thresholds_and_metric_scores);
    if (mm.max_criteria_and_metric_scores) add(prefix + " - Maximum metrics", mm.max_criteria_and_metric_scores);
    if (mm.gains_lift_table) add(prefix + " - Gains/Lift table", mm.gains_lift_table);
  };
  switch (res.kind) {
    case "model": {
      out.push({ name: "parameters", columns: ["parameter", "value", "default"],
        rows: (d.parameters || []).map((p) => [p.name, JSON.stringify(keyName(p.actual_value)), JSON.stringify(keyName(p.default_value))]) });
      const o = d.output || {};
      for (const [k, v] of Object.entries(o)) {
        if (v && v.columns && v.data) add("output - " + (v.name || k), v);
      }
      metrics("output - training_metrics", o.training_metrics);
      metrics("output - validation_metrics", o.validation_metrics);
      metrics("output - cross_validation_metrics", o.cross_validation_metrics);
      break;
    }
    case "prediction": for (const mm of d.model_metrics || []) metrics("prediction", mm); break;
    case "grid": if (d.summary_table) add("summary", d.summary_table); break;
    case "leaderboard": if (d.table) add("leaderboard", d.table); break;
    case "frameSummary": out.push({ name: "columns", columns: ["column", "type", "missing", "min", "max", "mean", "sigma"],
      rows: (d.columns || []).map((c) => [c.label, c.type, c.missing_count, (c.mins || [])[0], (c.maxs || [])[0], c.mean, c.sigma]) }); break;
    case "table": out.push(d); break;
    case "tables": out.push(...d); break;
    default: break;
  }
  return out;
}

// ------------------------------------------------------------------------------------------------ rendering
const esc = (s) => String(s === null || s === undefined ? "" : s).replace(/[&<>"]/g,
  (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;" })[c]);
const fmt = (v) => (typeof v === "number" && !Number.isInteger(v) ? Number(v.toPrecision(6)) : v);

function table(cols, rows) {
  return "<table><thead><tr>" + cols.map((c) => "<th>" + esc(c) + "</th>").join("") + "</tr></thead><tbody>" +
    rows.map((r) => "<tr>" + r.map((v) => "<td>" + esc(fmt(v)) + "</td>").join("") + "</tr>").join("") +
    "</tbody></table>";
}

// TwoDimTableV3: columns [{name}], data column-major
function twoDim(t) {
  if (!t || !t.columns) return "";
  const r = twoDimRows(t);
  return "<h4>" + esc(r.name) + "</h4>" + table(r.columns, r.rows);
}

function metricsHtml(mm) {
  if (!mm) return "";
  const keys = ["MSE", "RMSE", "logloss", "AUC", "pr_auc", "mean_per_class_error", "r2", "mean_residual_deviance"];
  const rows = keys.filter((k) => mm[k] !== undefined && mm[k] !== null).map((k) => [k, mm[k]]);
  return table(["metric", "value"], rows) + (mm.cm && mm.cm.table ? twoDim(mm.cm.table) : "");
}

// markdown cells: headings, emphasis, code, links, lists — text is escaped first (no raw HTML from notebooks)
function markdown(src) {
  const inline = (s) => esc(s)
    .replace(/`([^`]+)`/g, "<code>$1</code>")
    .replace(/\*\*([^*]+)\*\*/g, "<b>$1</b>")
    .replace(/\*([^*]+)\*/g, "<i>$1</i>")
    .replace(/\[([^\]]+)\]\((https?:[^)\s]+)\)/g, (m, t, u) => '<a href="' + u + '" rel="noopener" target="_blank">' + t + "</a>");
  const out = [];
  let list = null;
  for (const line of String(src || "").split("\n")) {
    const h = /^(#{1,6})\s+(.*)$/.exec(line);
    const li = /^\s*(?:[-*]|\d+\.)\s+(.*)$/.exec(line);
    if (li) { if (!list) { list = []; } list.push("<li>" + inline(li[1]) + "</li>"); continue; }
    if (list) { out.push("<ul>" + list.join("") + "</ul>"); list = null; }
    if (h) out.push("<h" + h[1].length + ">" + inline(h[2]) + "</h" + h[1].length + ">");
    else if (line.trim()) out.push("<p>" + inline(line) + "</p>");
  }
  if (list) out.push("<ul>" + list.join("") + "</ul>");
  return out.join("");
}

function render(res) {
  const d = res.data;
  switch (res.kind) {
    case "text": return "<p>" + esc(d) + "</p>";
    case "help": return table(["command", "description"], d.map((r) => [r.command, r.description]));
    case "assist": return "<p>" + esc(d.routine) + ": " + esc(d.doc) + "</p>" +
      (d.algos ? table(["algo"], d.algos.map((a) => [a])) : "") +
      (d.args && d.args.length ? "<pre>" + esc(JSON.stringify(d.args)) + "</pre>" : "");
    case "form": return "<p>" + esc(d.routine) + " needs " + esc((d.needs || []).join(", ")) + "</p>" +
      (d.frames ? table(["frame"], d.frames.map((f) => [f])) : "");
    case "markdown": {
      const hm = /^h([1-6])$/.exec(d.type || "");
      if (hm) return "<h" + hm[1] + ">" + esc(d.input) + "</h" + hm[1] + ">";
      if (d.type === "raw") return "<pre>" + esc(d.input) + "</pre>";
      return markdown(d.input);
    }
    case "cloud": return "<p>" + esc(d.cloud_name) + ": " + esc(d.cloud_size) + " node(s), version " + esc(d.version) +
      "</p>" + table(["node", "healthy"], (d.nodes || []).map((n) => [n.h2o || n.ip_port, n.healthy]));
    case "frames": return table(["frame", "rows", "columns"], d.map((f) => [keyName(f.frame_id), f.rows, f.columns ||
      f.num_columns]));
    case "frameSummary": return "<h3>" + esc(keyName(d.frame_id)) + "</h3><p>" + esc(d.rows) + " rows</p>" +
      table(["column", "type", "missing", "min", "max", "mean", "sigma", "cardinality"], (d.columns || []).map((c) =>
        [c.label, c.type, c.missing_count, (c.mins || [])[0], (c.maxs || [])[0], c.mean, c.sigma,
          c.domain ? c.domain.length : ""]));
    case "frameData": {
      const cols = d.columns || [];
      const n = cols.length ? (cols[0].data || cols[0].string_data || []).length : 0;
      const rows = [];
      for (let i = 0; i < n; i++) rows.push(cols.map((c) => {
        if (c.domain && c.data) return c.data[i] === null ? "" : c.domain[c.data[i]];
        return (c.string_data || c.data)[i];
      }));
      return table(cols.map((c) => c.label), rows);
    }
    case "import": return table(["file"], (d.files || []).map((f) => [f])) +
      (d.fails && d.fails.length ? "<p>failed: " + esc(d.fails.join(", ")) + "</p>" : "");
    case "parseSetup": return "<p>destination " + esc(d.destination_frame) + "</p>" +
      table(["column", "type"], (d.column_names || []).map((c, i) => [c, (d.column_types || [])[i]]));
    case "split": return table(["frame"], (d.destination_frames || []).map((f) => [keyName(f)]));
    case "models": return table(["model", "algo", "response"], d.map((m) => [keyName(m.model_id), m.algo,
      m.response_column_name || ""]));
    case "model": {
      const o = d.output || {};
      return "<h3>" + esc(keyName(d.model_id)) + " (" + esc(d.algo) + ")</h3>" +
        (o.model_summary ? twoDim(o.model_summary) : "") +
        (o.training_metrics ? "<h4>training metrics</h4>" + metricsHtml(o.training_metrics) : "") +
        (o.validation_metrics ? "<h4>validation metrics</h4>" + metricsHtml(o.validation_metrics) : "") +
        (o.variable_importances ? twoDim(o.variable_importances) : "");
    }
    case "prediction": return "<p>predictions: " + esc(keyName(d.predictions_frame) ||
      keyName(((d.model_metrics || [])[0] || {}).frame)) + "</p>" +
      ((d.model_metrics || []).length ? metricsHtml(d.model_metrics[0]) : "");
    case "grids": return table(["grid", "models"], d.map((g) => [keyName(g.grid_id), (g.model_ids || []).length]));
    case "grid": return "<h3>" + esc(keyName(d.grid_id)) + "</h3>" + (d.summary_table ? twoDim(d.summary_table) : "");
    case "table": return "<h4>" + esc(d.name) + "</h4>" + table(d.columns, d.rows);
    case "tables": return d.map((t) => "<h4>" + esc(t.name) + "</h4>" + table(t.columns, t.rows)).join("");
    case "jobs": return table(["job", "description", "status", "progress", "dest"], d.map((j) =>
      [keyName(j.key), j.description, j.status, j.progress, keyName(j.dest)]));
    case "leaderboard": return twoDim(d.table);
    case "builders": return table(["algo"], d.map((a) => [a]));
    case "notebook": return table(["#", "type", "cell"], (d.cells || []).map((c, i) => [i + 1, c.type, c.input]));
    default: return "<pre>" + esc(JSON.stringify(d, null, 1)) + "</pre>";
  }
}

const Flow = { parseCell, toJSON, runCell, runCommand, render, markdown, tablesOf, toFlowDoc, fromFlowDoc, COMMANDS,
  waitJob };
if (typeof module !== "undefined" && module.exports) module.exports = Flow;
if (typeof window !== "undefined") window.Flow = Flow;
