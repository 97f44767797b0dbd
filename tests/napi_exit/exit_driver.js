'use strict';
// Exit-path driver for fmt_napi.node over the CPU stub libfmt (tests/napi_exit/fmt_stub.cpp; TEST
// INFRASTRUCTURE). One run: the main thread opens engine contexts, runs async replays (one still
// pending when the process exits), closes some and leaves some open for the env cleanup hook;
// worker_threads open their own contexts, one hands its handle to the main thread (which must be
// refused: a context belongs to the env that opened it), and each worker's teardown must close only
// its own contexts (the main thread's still replay afterwards). Garbage and forced GCs run between
// steps so weak-callback passes, if any handle had one, would be queued when the environment is torn
// down. Prints "exit-driver ok" and exits 0, or throws.
const path = require('path');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');

const addon = require(process.env.FMT_NAPI_ADDON || path.join(__dirname, '..', '_build', 'napi_exit', 'fmt_napi.node'));
const OP = addon.sizes.mtOp;

function batch(nDocs, opsPerDoc) {
  const offs = new BigUint64Array(nDocs + 1);
  for (let d = 0; d <= nDocs; d++) offs[d] = BigInt(d * opsPerDoc);
  return {
    ops: new Uint8Array(nDocs * opsPerDoc * OP),
    docOpOffsets: offs,
    text: new Uint16Array(16),
    docInit: new Uint32Array(nDocs * 2),
    propsOff: new Uint32Array(1),
    propsKv: new Uint32Array(0),
  };
}

function churn() {  // garbage for the GC, plus a forced collection when --expose-gc
  let keep = [];
  for (let i = 0; i < 2000; i++) keep.push({ a: new Array(32).fill(i), b: 'x' + i });
  keep = null;
  if (global.gc) global.gc();
}

async function replayOnce(ctx, nDocs) {
  const hdrs = await addon.replayMergeTree(ctx, batch(nDocs, 4));
  if (!(hdrs instanceof ArrayBuffer) || hdrs.byteLength !== nDocs * addon.sizes.docResult) throw new Error('bad headers');
}

function expectUsage(fn, what) {
  try {
    fn();
  } catch (e) {
    if (e.code === 'FMT_E_USAGE' && (!what || String(e.message).includes(what))) return;
    throw e;
  }
  throw new Error('expected FMT_E_USAGE' + (what ? ' (' + what + ')' : ''));
}

async function workerMain() {
  const ctx = addon.open(0);
  await replayOnce(ctx, 3);
  churn();
  if (workerData.handOver) {
    parentPort.postMessage({ handle: ctx });
    await new Promise((res) => parentPort.once('message', res));  // main has tried it
  }
  if (workerData.close) addon.close(ctx);
  parentPort.postMessage({ done: true });
}

async function main() {
  const rounds = Number(process.env.EXIT_ROUNDS || 3);
  const mine = addon.open(0);
  for (let r = 0; r < rounds; r++) {
    const a = addon.open(0), b = addon.open(0);
    await Promise.all([replayOnce(a, 5), replayOnce(b, 2)]);
    churn();
    addon.close(a);
    expectUsage(() => addon.deviceInfo(a), 'closed');  // stale handle: detected, never dereferenced
    addon.close(a);  // closing twice is a no-op
    // b stays open: the env cleanup hook closes it at teardown
  }
  // workers: each opens its own context; one hands its handle over while it is alive
  const workers = [];
  for (let w = 0; w < (process.env.EXIT_NO_WORKERS ? 0 : 4); w++) {
    workers.push(new Promise((resolve, reject) => {
      const wk = new Worker(__filename, { workerData: { handOver: w === 0, close: w % 2 === 1 } });
      wk.on('message', (m) => {
        if (m.handle !== undefined) {
          expectUsage(() => addon.deviceInfo(m.handle), 'another thread');
          expectUsage(() => addon.close(m.handle), 'another thread');
          wk.postMessage('tried');
        }
      });
      wk.on('error', reject);
      wk.on('exit', (code) => (code === 0 ? resolve() : reject(new Error('worker exit ' + code))));
    }));
  }
  await Promise.all(workers);
  churn();
  // the workers' teardown closed only their own contexts: the main thread's still work
  await replayOnce(mine, 7);
  if (typeof addon.deviceInfo(mine) !== 'string') throw new Error('deviceInfo');
  // leave one replay pending at exit (its context busy: left to process exit by the cleanup hook)
  const pend = addon.open(0);
  addon.replayMergeTree(pend, batch(64, 64)).catch(() => {});
  churn();
  // many dead handles, then garbage without a forced collection: a natural GC's weak-callback second
  // pass (if any handle had a weak reference) is then still queued when the environment is torn down
  const nHandles = Number(process.env.EXIT_HANDLES || 2000);
  for (let i = 0; i < nHandles; i++) addon.close(addon.open(0));
  let junk = [];
  for (let i = 0; i < 200000; i++) junk.push({ i, s: 'y' + i });
  junk = null;
  console.log('exit-driver ok', addon.openContexts());
}

if (isMainThread) {
  main().catch((e) => {
    console.error(e && e.stack ? e.stack : e);
    process.exit(1);
  });
} else {
  workerMain().catch((e) => {
    console.error(e && e.stack ? e.stack : e);
    process.exit(2);
  });
}
