"use strict";
/**
 * oracle/js/mt_observer.js — CPU BASELINE ONLY (a JS restatement, not the reference, and not the
 * product path): the SharedString observer path in plain JavaScript on worker_threads, over the
 * flat op records of include/fmt.h (fmt_mt_op, 32 B).
 *
 * A document is a flat list of segments {text, ins seq, ins client, removes [[seq, client]...],
 * props}; a remote op resolves its positions in PriorPerspective(refSeq, client) (perspective.ts:
 * 80-93: a stamp has occurred if seq <= refSeq or it is the op's own client) and then:
 *   insert  mergeTree.ts:1811-1987 insertingWalk, flattened: the first segment where the position
 *           falls strictly inside (split) or, at a segment start, that has length there or wins
 *           breakTie (:1890-1905: the new op is newer than its insert, or its first remove is
 *           newer than the op);
 *   remove  mergeTree.ts:2297-2382 markRangeRemoved: boundaries split, every segment of positive
 *           length in [pos1, pos2) gets the remove stamp (the first one removes it);
 *   annotate mergeTree.ts:2009-2081 + segmentPropertiesManager.ts:188-238 (raw LWW; null deletes).
 * Segments removed at or below minSeq are dropped (zamboni without the merges: it changes no
 * visible text). The B+tree and partial lengths of the reference are not restated — this is the
 * plain-JS cost of the observer semantics, which tests/test_js_baseline.py pins by each document's
 * final visible text against the C++ oracle's.
 *
 * Usage: node mt_observer.js <dir> <workers> [reps]   (dir: ops.bin offs.bin text.bin init.bin
 *        props_off.bin props_kv.bin meta.json {keys, values}; writes hashes.bin = FNV-1a of each
 *        document's final text, UTF-16 units)
 * Prints one JSON line {docs, ops, workers, reps, seconds, ops_per_s}.
 * Written for the Node in this image (v12): CommonJS, no `??` / `?.`.
 */
const fs = require("fs");
const path = require("path");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");

const INSERT = 0, REMOVE = 1, ANNOTATE = 2;

function textOf(text, off, len) {
  let s = "";
  for (let i = 0; i < len; i += 4096) s += String.fromCharCode.apply(null, text.subarray(off + i, off + Math.min(len, i + 4096)));
  return s;
}

function replayDoc(I, d) {
  const ops = I.ops, u = I.opsU;
  const segs = [];
  if (I.init[2 * d + 1] > 0) segs.push({ text: textOf(I.text, I.init[2 * d], I.init[2 * d + 1]), ins: 0, client: -1, rm: null, props: null });
  let minSeq = 0;
  const present = (s, r, c) => {
    if (!(s.ins <= r || s.client === c)) return false;
    if (s.rm !== null) for (let k = 0; k < s.rm.length; k += 2) if (s.rm[k] <= r || s.rm[k + 1] === c) return false;
    return true;
  };
  const split = (i, at) => {
    const s = segs[i];
    const t = { text: s.text.slice(at), ins: s.ins, client: s.client, rm: s.rm === null ? null : s.rm.slice(),
      props: s.props === null ? null : Object.assign({}, s.props) };
    s.text = s.text.slice(0, at);
    segs.splice(i + 1, 0, t);
  };
  // split so that a segment starts at perspective position pos (ensureIntervalBoundary)
  const boundary = (pos, r, c) => {
    let rem = pos;
    for (let i = 0; i < segs.length; i++) {
      const len = present(segs[i], r, c) ? segs[i].text.length : 0;
      if (rem < len) {
        if (rem > 0) split(i, rem);
        return;
      }
      rem -= len;
    }
  };
  const range = (p1, p2, r, c, fn) => {
    boundary(p1, r, c);
    boundary(p2, r, c);
    let pos = 0;
    for (let i = 0; i < segs.length && pos < p2; i++) {
      const len = present(segs[i], r, c) ? segs[i].text.length : 0;
      if (len === 0) continue;
      if (pos >= p1) fn(segs[i]);
      pos += len;
    }
  };
  for (let i = Number(I.offs[d]), e = Number(I.offs[d + 1]); i < e; i++) {
    const seq = ops[8 * i], r = ops[8 * i + 1], msn = ops[8 * i + 2], p1 = ops[8 * i + 3], p2 = ops[8 * i + 4];
    const w6 = u[8 * i + 6], type = w6 >>> 24, c = (w6 >>> 16) & 0xff;
    if (type === INSERT) {
      const seg = { text: textOf(I.text, u[8 * i + 5], w6 & 0xffff), ins: seq, client: c, rm: null, props: null };
      let rem = p1, at = segs.length;
      for (let k = 0; k < segs.length; k++) {
        const s = segs[k];
        const len = present(s, r, c) ? s.text.length : 0;
        if (rem < len) {
          if (rem > 0) {
            split(k, rem);
            at = k + 1;
          } else at = k;
          break;
        }
        if (rem === 0 && (seq > s.ins || (s.rm !== null && s.rm[0] > seq))) {
          at = k;
          break;
        }
        rem -= len;
      }
      segs.splice(at, 0, seg);
    } else if (type === REMOVE) {
      if (p2 > p1) range(p1, p2, r, c, (s) => {
        if (s.rm === null) s.rm = [seq, c];
        else s.rm.push(seq, c);
      });
    } else if (type === ANNOTATE) {
      const pid = u[8 * i + 5];
      const k0 = I.propsOff[pid], k1 = I.propsOff[pid + 1];
      if (p2 > p1) range(p1, p2, r, c, (s) => {
        if (s.props === null) s.props = {};
        for (let k = k0; k < k1; k++) {
          const kv = I.propsKv[k], key = I.keys[kv >>> 16], v = kv & 0xffff;
          if (v === 0) delete s.props[key];
          else s.props[key] = I.values[v];
        }
      });
    } else {
      throw new Error("op type " + type + " is not restated here");
    }
    if (msn > minSeq) {  // zamboni, minus the merges: segments removed at or below minSeq go
      minSeq = msn;
      for (let k = segs.length - 1; k >= 0; k--) if (segs[k].rm !== null && segs[k].rm[0] <= minSeq) segs.splice(k, 1);
    }
  }
  let h = 0x811c9dc5;
  for (const s of segs) {
    if (s.rm !== null) continue;
    for (let k = 0; k < s.text.length; k++) h = Math.imul(h ^ s.text.charCodeAt(k), 16777619) >>> 0;
  }
  return h;
}

function views(sabs, meta) {
  return {
    ops: new Int32Array(sabs.ops), opsU: new Uint32Array(sabs.ops), offs: new BigUint64Array(sabs.offs),
    text: new Uint16Array(sabs.text), init: new Uint32Array(sabs.init), propsOff: new Uint32Array(sabs.propsOff),
    propsKv: new Uint32Array(sabs.propsKv), keys: meta.keys, values: meta.values,
  };
}

if (isMainThread) {
  const [dir, workersArg, repsArg] = process.argv.slice(2);
  const reps = Math.max(1, parseInt(repsArg || "1", 10));
  const load = (f) => {
    const b = fs.readFileSync(path.join(dir, f));
    const sab = new SharedArrayBuffer(Math.max(8, b.length));
    Buffer.from(sab).set(b);
    return sab;
  };
  const sabs = { ops: load("ops.bin"), offs: load("offs.bin"), text: load("text.bin"), init: load("init.bin"),
    propsOff: load("props_off.bin"), propsKv: load("props_kv.bin") };
  const meta = JSON.parse(fs.readFileSync(path.join(dir, "meta.json"), "utf8"));
  const nDocs = fs.statSync(path.join(dir, "offs.bin")).size / 8 - 1;
  const hashSab = new SharedArrayBuffer(4 * Math.max(1, nDocs));
  const W = Math.max(1, parseInt(workersArg, 10));
  let ready = 0, done = 0, t0 = 0;
  const workers = [];
  for (let w = 0; w < W; w++) {
    const wk = new Worker(__filename, { workerData: { sabs, meta, hashSab, nDocs, first: w, step: W, reps } });
    wk.on("message", (m) => {
      if (m === "ready" && ++ready === W) {
        t0 = process.hrtime.bigint();
        workers.forEach((x) => x.postMessage("go"));
      } else if (m === "done" && ++done === W) {
        const secs = Number(process.hrtime.bigint() - t0) / 1e9;
        const nOps = Number(new BigUint64Array(sabs.offs)[nDocs]) * reps;
        fs.writeFileSync(path.join(dir, "hashes.bin"), Buffer.from(hashSab, 0, 4 * nDocs));
        console.log(JSON.stringify({ docs: nDocs, ops: nOps, workers: W, reps: reps, seconds: secs, ops_per_s: nOps / secs }));
        workers.forEach((x) => x.terminate());
      }
    });
    wk.on("error", (err) => {
      console.error(err);
      process.exit(1);
    });
    workers.push(wk);
  }
} else {
  const { sabs, meta, hashSab, nDocs, first, step, reps } = workerData;
  const I = views(sabs, meta);
  const hashes = new Uint32Array(hashSab);
  parentPort.on("message", () => {
    for (let r = 0; r < reps; r++) for (let d = first; d < nDocs; d += step) hashes[d] = replayDoc(I, d);
    parentPort.postMessage("done");
  });
  parentPort.postMessage("ready");
}
