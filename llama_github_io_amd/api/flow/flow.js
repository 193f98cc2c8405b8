// Flow: the notebook web UI of the REST server (reference: h2o-web / h2o-flow, served at /flow/index.html).
//
// A Flow notebook is a list of cells; a cell holds one command in Flow's routine syntax
// (`getFrames`, `importFiles ["data.csv"]`, `buildModel "gbm", {training_frame: "f", ...}`, ...). This file is
// the whole command layer: parsing a cell (parseCell), running it against the REST API (runCell, with an
// injected `http(method, path, body)` so the same code runs in the browser and under node in the tests), and
// rendering the result as HTML (render). index.html is only the page shell around it.
"use strict";

// ------------------------------------------------------------------------------------------------ parsing
// Flow's routines take CoffeeScript arguments; cells here take the JSON subset Flow users write:
// strings, numbers, booleans, null, arrays and objects whose keys may be bare identifiers, and a bare
// `key: value, ...` list as one object argument (`predict model: "m", frame: "f"`).
function toJSON(src) {
  let out = "", i = 0;
  while (i < src.length) {
    const c = src[i];
    if (c === '"' || c === "'") {                       // string literal (single quotes -> double)
      let j = i + 1, s = "";
      while (j < src.length && src[j] !== c) {
        if (src[j] === "\\" && j + 1 < src.length) { s += src[j] + src[j + 1]; j += 2; continue; }
        if (c === "'" && src[j] === '"') { s += '\\"'; j++; continue; }
        s += src[j++];
      }
      if (j >= src.length) throw new Error("unterminated string");
      out += '"' + s + '"';
      i = j + 1;
      continue;
    }
    const m = /^[A-Za-z_$][\w$]*/.exec(src.slice(i));
    if (m) {
      const w = m[0], rest = src.slice(i + w.length);
      if (/^\s*:/.test(rest)) out += '"' + w + '"';    // bare object key
      else if (w === "true" || w === "false" || w === "null") out += w;
      else if (w === "undefined") out += "null";
      else throw new Error("unexpected identifier " + w);
      i += w.length;
      continue;
    }
    out += c;
    i++;
  }
  return out;
}

function parseCell(text) {
  const src = String(text || "").trim().replace(/;\s*$/, "");
  if (!src) return null;
  const m = /^([A-Za-z_][\w]*)\s*(.*)$/s.exec(src);
  if (!m) throw new Error("a cell starts with a command name");
  const name = m[1];
  let rest = m[2].trim();
  if (rest.startsWith("(") && rest.endsWith(")")) rest = rest.slice(1, -1).trim();
  if (!rest) return { name, args: [] };
  // `key: value, ...` without braces is one object argument
  if (/^[A-Za-z_$][\w$]*\s*:/.test(rest)) rest = "{" + rest + "}";
  let args;
  try {
    args = JSON.parse("[" + toJSON(rest) + "]");
  } catch (e) {
    throw new Error("cannot parse the arguments of " + name + ": " + e.message);
  }
  return { name, args };
}

// ------------------------------------------------------------------------------------------------ commands
const enc = encodeURIComponent;
const keyName = (k) => (k && typeof k === "object" ? k.name : k);

async function waitJob(http, job, opts) {
  const key = keyName(job.key);
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

const COMMANDS = {
  help: { doc: "list the commands", run: async () => ({ kind: "help", data: Object.keys(COMMANDS).sort().map(
    (k) => ({ command: k, description: COMMANDS[k].doc })) }) },
  getCloud: { doc: "cluster status", run: async (h) => ({ kind: "cloud", data: await h("GET", "/3/Cloud") }) },
  getTimeline: { doc: "recent REST events", run: async (h) => ({ kind: "json", data: await h("GET", "/3/Timeline") }) },
  getFrames: { doc: "list frames", run: async (h) => ({ kind: "frames", data: (await h("GET", "/3/Frames")).frames }) },
  getFrameSummary: { doc: 'getFrameSummary "frame": column summaries',
    run: async (h, [f]) => ({ kind: "frameSummary", data: (await h("GET", "/3/Frames/" + enc(f) + "/summary")).frames[0] }) },
  getFrameData: { doc: 'getFrameData "frame": the first rows',
    run: async (h, [f, n]) => ({ kind: "frameData",
      data: (await h("GET", "/3/Frames/" + enc(f) + "?row_count=" + (n || 10))).frames[0] }) },
  deleteFrame: { doc: 'deleteFrame "frame"',
    run: async (h, [f]) => { await h("DELETE", "/3/Frames/" + enc(f)); return { kind: "text", data: "deleted frame " + f }; } },
  importFiles: { doc: 'importFiles ["path", ...]: register files for parsing',
    run: async (h, [paths]) => ({ kind: "import",
      data: await h("POST", "/3/ImportFilesMulti", { paths: Array.isArray(paths) ? paths : [paths] }) }) },
  setupParse: { doc: 'setupParse source_frames: ["path"]: guess the parse setup',
    run: async (h, [o]) => ({ kind: "parseSetup", data: await h("POST", "/3/ParseSetup", o) }) },
  parseFiles: { doc: "parseFiles {source_frames, destination_frame, ...}: parse into a frame",
    run: async (h, [o], opts) => {
      const r = await h("POST", "/3/Parse", o);
      await waitJob(h, r.job, opts);
      const f = keyName(r.destination_frame);
      return { kind: "frameSummary", data: (await h("GET", "/3/Frames/" + enc(f) + "/summary")).frames[0] };
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
  splitFrame: { doc: 'splitFrame "frame", [0.75], ["train", "test"]',
    run: async (h, [f, ratios, dests, seed]) => ({ kind: "json", data: await h("POST", "/3/SplitFrame",
      { dataset: f, ratios: ratios || [0.75], destination_frames: dests, seed: seed === undefined ? null : seed }) }) },
  getModels: { doc: "list models", run: async (h) => ({ kind: "models", data: (await h("GET", "/3/Models")).models }) },
  getModel: { doc: 'getModel "model"',
    run: async (h, [m]) => ({ kind: "model", data: (await h("GET", "/3/Models/" + enc(m))).models[0] }) },
  deleteModel: { doc: 'deleteModel "model"',
    run: async (h, [m]) => { await h("DELETE", "/3/Models/" + enc(m)); return { kind: "text", data: "deleted model " + m }; } },
  getModelBuilders: { doc: "algorithms that can be built",
    run: async (h) => ({ kind: "builders", data: Object.keys((await h("GET", "/3/ModelBuilders")).model_builders).sort() }) },
  buildModel: { doc: 'buildModel "gbm", {training_frame: "f", response_column: "y", ...}',
    run: async (h, [algo, params], opts) => {
      const r = await h("POST", "/3/ModelBuilders/" + enc(algo), params || {});
      const j = await waitJob(h, r.job, opts);
      return { kind: "model", data: (await h("GET", "/3/Models/" + enc(keyName(j.dest)))).models[0] };
    } },
  predict: { doc: 'predict model: "m", frame: "f" [, predictions_frame: "p"]',
    run: async (h, [o]) => ({ kind: "prediction", data: await h("POST", "/3/Predictions/models/" + enc(o.model) +
      "/frames/" + enc(o.frame), o.predictions_frame ? { predictions_frame: o.predictions_frame } : {}) }) },
  getJobs: { doc: "list jobs", run: async (h) => ({ kind: "jobs", data: (await h("GET", "/3/Jobs")).jobs }) },
  getJob: { doc: 'getJob "job"', run: async (h, [k]) => ({ kind: "jobs", data: (await h("GET", "/3/Jobs/" + enc(k))).jobs }) },
  cancelJob: { doc: 'cancelJob "job"',
    run: async (h, [k]) => { await h("POST", "/3/Jobs/" + enc(k) + "/cancel"); return { kind: "text", data: "cancelled " + k }; } },
  runAutoML: { doc: 'runAutoML {training_frame: "f", response_column: "y", max_models: 5, project_name: "p"}',
    run: async (h, [o], opts) => {
      o = o || {};
      const spec = { input_spec: { training_frame: o.training_frame, response_column: o.response_column,
          validation_frame: o.validation_frame, leaderboard_frame: o.leaderboard_frame, ignored_columns: o.ignored_columns },
        build_control: { project_name: o.project_name, nfolds: o.nfolds === undefined ? 5 : o.nfolds,
          stopping_criteria: { max_models: o.max_models, max_runtime_secs: o.max_runtime_secs, seed: o.seed } },
        build_models: { include_algos: o.include_algos, exclude_algos: o.exclude_algos } };
      const r = await h("POST", "/99/AutoMLBuilder", spec);
      await waitJob(h, r.job, opts);
      const pid = r.build_control.project_name;
      return { kind: "leaderboard", data: await h("GET", "/99/Leaderboards/" + enc(pid)) };
    } },
  getLeaderboard: { doc: 'getLeaderboard "project"',
    run: async (h, [p]) => ({ kind: "leaderboard", data: await h("GET", "/99/Leaderboards/" + enc(p)) }) },
  runRapids: { doc: 'runRapids "(expression)": evaluate a Rapids expression',
    run: async (h, [ast]) => ({ kind: "json", data: await h("POST", "/99/Rapids", { ast, session_id: "_flow" }) }) },
  saveFlow: { doc: 'saveFlow "name": store this notebook on the server',
    run: async (h, [name], opts) => {
      const cells = (opts && opts.cells) || [];
      await h("POST", "/3/NodePersistentStorage/notebook/" + enc(name), { value: JSON.stringify({ version: 1, cells }) });
      return { kind: "text", data: "saved notebook " + name + " (" + cells.length + " cells)" };
    } },
  loadFlow: { doc: 'loadFlow "name": the cells of a stored notebook',
    run: async (h, [name]) => {
      const r = await h("GET", "/3/NodePersistentStorage/notebook/" + enc(name));
      return { kind: "notebook", data: JSON.parse(r.value) };
    } },
  getFlows: { doc: "stored notebooks",
    run: async (h) => ({ kind: "json", data: (await h("GET", "/3/NodePersistentStorage/notebook")).entries }) },
};

async function runCell(http, text, opts) {
  const c = parseCell(text);
  if (!c) return { kind: "text", data: "" };
  const cmd = COMMANDS[c.name];
  if (!cmd) throw new Error("unknown command " + c.name + " (try help)");
  return cmd.run(http, c.args, opts || {});
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
  const n = t.rowcount || (t.data && t.data[0] ? t.data[0].length : 0);
  const rows = [];
  for (let i = 0; i < n; i++) rows.push(t.data.map((col) => col[i]));
  return "<h4>" + esc(t.name || "") + "</h4>" + table(t.columns.map((c) => c.name), rows);
}

function metricsHtml(mm) {
  if (!mm) return "";
  const keys = ["MSE", "RMSE", "logloss", "AUC", "pr_auc", "mean_per_class_error", "r2", "mean_residual_deviance"];
  const rows = keys.filter((k) => mm[k] !== undefined && mm[k] !== null).map((k) => [k, mm[k]]);
  return table(["metric", "value"], rows) + (mm.cm && mm.cm.table ? twoDim(mm.cm.table) : "");
}

function render(res) {
  const d = res.data;
  switch (res.kind) {
    case "text": return "<p>" + esc(d) + "</p>";
    case "help": return table(["command", "description"], d.map((r) => [r.command, r.description]));
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
    case "prediction": return "<p>predictions: " + esc(keyName(d.predictions_frame)) + "</p>" +
      ((d.model_metrics || []).length ? metricsHtml(d.model_metrics[0]) : "");
    case "jobs": return table(["job", "description", "status", "progress", "dest"], d.map((j) =>
      [keyName(j.key), j.description, j.status, j.progress, keyName(j.dest)]));
    case "leaderboard": return twoDim(d.table);
    case "builders": return table(["algo"], d.map((a) => [a]));
    case "notebook": return table(["#", "cell"], (d.cells || []).map((c, i) => [i + 1, c]));
    default: return "<pre>" + esc(JSON.stringify(d, null, 1)) + "</pre>";
  }
}

const Flow = { parseCell, toJSON, runCell, render, COMMANDS, waitJob };
if (typeof module !== "undefined" && module.exports) module.exports = Flow;
if (typeof window !== "undefined") window.Flow = Flow;
