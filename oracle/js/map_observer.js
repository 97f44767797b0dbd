"use strict";
/**
 * oracle/js/map_observer.js — CPU BASELINE ONLY (a JS restatement, not the reference, and not the
 * product path): the SharedMap observer path in plain JavaScript, run on worker_threads.
 *
 * What a Fluid client does with each sequenced remote map op, restated over the flat op records of
 * include/fmt.h (fmt_map_op, 16 B: doc, key id, seq, kind << 30 | value id):
 *   "set"    mapKernel.ts:802-850  sequencedData.set(key, localValue)   (existing key keeps its place)
 *   "delete" mapKernel.ts:761-801  sequencedData.delete(key)
 *   "clear"  mapKernel.ts:708-760  sequencedData.clear()
 * on a real JS Map keyed by the key STRING, as the reference's MapKernel is. Each document's final
 * Map is folded into a 32-bit hash of its entries in iteration order, (key id, value id) per entry,
 * which tests/test_js_baseline.py checks against the C++ oracle's entries.
 *
 * Usage: node map_observer.js <ops.bin> <offsets.bin (u64, n_docs + 1)> <keys.json> <workers> <out hashes.bin> [reps]
 * Prints one JSON line {docs, ops, workers, reps, seconds, ops_per_s}: seconds = from the moment
 * every worker holds its inputs until the last worker finishes its `reps` passes over them (the
 * inputs are shared, not copied); ops counts every pass.
 * Written for the Node in this image (v12): CommonJS, no `??` / `?.`.
 */
const fs = require("fs");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");

const MAP_DELETE = 1, MAP_CLEAR = 2, KIND_SHIFT = 30, VALUE_MASK = 0x3fffffff;

function replayDocs(ops, offs, keys, hashes, first, step) {
  const nDocs = hashes.length;
  for (let d = first; d < nDocs; d += step) {
    const data = new Map();
    const b = Number(offs[d]), e = Number(offs[d + 1]);
    for (let i = b; i < e; i++) {
      const kv = ops[4 * i + 3];
      const kind = kv >>> KIND_SHIFT;
      if (kind === MAP_CLEAR) {
        data.clear();
      } else if (kind === MAP_DELETE) {
        data.delete(keys[ops[4 * i + 1]]);
      } else {
        data.set(keys[ops[4 * i + 1]], { id: ops[4 * i + 1], value: kv & VALUE_MASK });
      }
    }
    let h = 0x811c9dc5;
    data.forEach((v) => {
      h = Math.imul(h ^ v.id, 16777619) >>> 0;
      h = Math.imul(h ^ v.value, 16777619) >>> 0;
    });
    hashes[d] = h;
  }
}

if (isMainThread) {
  const [opsPath, offsPath, keysPath, workersArg, outPath, repsArg] = process.argv.slice(2);
  const reps = Math.max(1, parseInt(repsArg || "1", 10));
  const opsBuf = fs.readFileSync(opsPath), offsBuf = fs.readFileSync(offsPath);
  const opsSab = new SharedArrayBuffer(opsBuf.length), offsSab = new SharedArrayBuffer(offsBuf.length);
  Buffer.from(opsSab).set(opsBuf);
  Buffer.from(offsSab).set(offsBuf);
  const nDocs = offsBuf.length / 8 - 1;
  const hashSab = new SharedArrayBuffer(4 * nDocs);
  const keys = JSON.parse(fs.readFileSync(keysPath, "utf8"));
  const W = Math.max(1, parseInt(workersArg, 10));
  let ready = 0, done = 0, t0 = 0;
  const workers = [];
  for (let w = 0; w < W; w++) {
    const wk = new Worker(__filename, { workerData: { opsSab, offsSab, hashSab, keys, first: w, step: W, reps } });
    wk.on("message", (m) => {
      if (m === "ready" && ++ready === W) {
        t0 = process.hrtime.bigint();
        workers.forEach((x) => x.postMessage("go"));
      } else if (m === "done" && ++done === W) {
        const secs = Number(process.hrtime.bigint() - t0) / 1e9;
        const nOps = Number(new BigUint64Array(offsSab)[nDocs]) * reps;
        fs.writeFileSync(outPath, Buffer.from(hashSab));
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
  const { opsSab, offsSab, hashSab, keys, first, step, reps } = workerData;
  const ops = new Uint32Array(opsSab), offs = new BigUint64Array(offsSab), hashes = new Uint32Array(hashSab);
  parentPort.on("message", () => {
    for (let r = 0; r < reps; r++) replayDocs(ops, offs, keys, hashes, first, step);
    parentPort.postMessage("done");
  });
  parentPort.postMessage("ready");
}
