"""Synthetic workloads of BASELINE.json's configs (ctypes over libfmtgen.so).

M1/M2: SharedMap fuzz-shaped LWW streams. T1/T2: merge-tree conflict-farm streams. See
csrc/gen/fmtgen.cpp for how each mirrors the reference's own stochastic generators.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from .streams import (MAP_OP_DTYPE, MT_ANNOTATE, MT_INSERT, MT_OP_DTYPE, MT_REMOVE, MT_SEG_MARKER, NO_PROPS, SNAPSHOT_DOC_DTYPE, SNAPSHOT_SEG_DTYPE, MapBatch,
                      MergeTreeBatch, js_json)

HERE = os.path.dirname(os.path.abspath(__file__))
GEN_PATH = os.path.join(HERE, "libfmtgen.so")
_gen = None


def _lib():
    global _gen
    if _gen is None:
        if not os.path.exists(GEN_PATH):
            subprocess.run(["make", "-s", "-C", os.path.join(HERE, "csrc", "gen")], check=True)
        L = ctypes.CDLL(GEN_PATH)
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.fmtgen_map.argtypes = [U32, U32, U32, U32, P, P, U32]
        L.fmtgen_conflict_farm_new.argtypes = [U32, U32, U32, U32, U32, U32, U32,
                                               ctypes.POINTER(U64), ctypes.POINTER(U64), U32]
        L.fmtgen_conflict_farm_new.restype = P
        L.fmtgen_conflict_farm_copy.argtypes = [P, U32, P, P, P, U32]
        L.fmtgen_free.argtypes = [P]
        L.fmtgen_t3.argtypes = [U32, U32, U32, U32, U32, U32, U32, P, P, P]
        L.fmtgen_t3.restype = ctypes.c_int64
        _gen = L
    return _gen


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def map_value_json(value_id: int) -> str:
    """JSON text of a synthetic map value id (ids < 50 are the integers 1..50)."""
    return str(value_id + 1) if value_id < 50 else js_json(f"s{value_id}")


def map_stream(n_docs: int, ops_per_doc: int, key_pool: int = 20, seed: int = 1, threads=None) -> MapBatch:
    ops = np.zeros(n_docs * ops_per_doc, dtype=MAP_OP_DTYPE)
    offs = np.zeros(n_docs + 1, dtype=np.uint64)
    rc = _lib().fmtgen_map(n_docs, ops_per_doc, key_pool, seed, _p(ops), _p(offs), threads or default_threads())
    if rc != 0:
        raise ValueError("fmtgen_map failed")
    keys = [str(k) for k in range(key_pool)]
    return MapBatch(ops=ops, doc_op_offsets=offs, key_bound=key_pool, keys=keys, values=_LazyValues())


class _LazyValues:
    """Value dictionary materialized on demand (string values are opaque synthetic ids)."""

    def __getitem__(self, i):
        return map_value_json(i)

    def __len__(self):
        return 0x3FFFFFFF


CLIENT_NAMES = [chr(ord("A") + i) for i in range(26)] + [chr(ord("a") + i) for i in range(26)] + [
    chr(ord("0") + i) for i in range(12)
] + [f"w{i}" for i in range(64, 254)]  # (short ids 64..253: the huge tier's writers)


def conflict_farm(n_docs: int, n_clients: int = 8, ops_per_doc: int = 2000, min_length: int = 0,
                  seed: int = 1, replicas: int = 1, threads=None, doc_base: int = 0) -> MergeTreeBatch:
    """Conflict-farm merge-tree streams; `replicas` lays out that many copies of the doc set.

    Documents are doc_base .. doc_base + n_docs - 1 of the seed's document set, so a shard of a big
    batch is generated alone with exactly the streams the whole batch would hold.
    Props op i is {"client": CLIENT_NAMES[i]} (the 0.40 fixtures' annotate shape).
    """
    L = _lib()
    threads = threads or default_threads()
    n_ops, n_text = ctypes.c_uint64(), ctypes.c_uint64()
    h = L.fmtgen_conflict_farm_new(n_docs, n_clients, ops_per_doc, min_length, seed, 0, threads,
                                   ctypes.byref(n_ops), ctypes.byref(n_text), doc_base)
    if not h:
        raise ValueError("fmtgen_conflict_farm_new failed")
    try:
        ops = np.zeros(n_ops.value * replicas, dtype=MT_OP_DTYPE)
        offs = np.zeros(n_docs * replicas + 1, dtype=np.uint64)
        text = np.zeros(max(1, n_text.value * replicas), dtype="<u2")
        rc = L.fmtgen_conflict_farm_copy(h, replicas, _p(ops), _p(offs), _p(text), threads)
        if rc != 0:
            raise ValueError(f"fmtgen_conflict_farm_copy failed ({rc})")
    finally:
        L.fmtgen_free(h)
    n_props = len(CLIENT_NAMES)
    props_off = np.arange(n_props + 1, dtype=np.uint32)
    values = ["null"] + [js_json(c) for c in CLIENT_NAMES]
    props_kv = np.array([(0 << 16) | (i + 1) for i in range(n_props)], dtype=np.uint32)
    return MergeTreeBatch(
        ops=ops,
        doc_op_offsets=offs,
        text=text,
        doc_init=np.zeros((n_docs * replicas, 2), dtype=np.uint32),
        props_off=props_off,
        props_kv=props_kv,
        keys=["client"],
        values=values,
    )


def t3_stream(n_segments: int = 10_000_000, n_ops: int = 10_000_000, n_clients: int = 63, max_lag: int = 4096,
              max_range: int = 8, seed: int = 1) -> MergeTreeBatch:
    """T3 (BASELINE.json config 5): one SharedString of n_segments segments loaded from a summary
    (one header chunk), then n_ops messages from n_clients writers with refSeq lag U[0, max_lag).
    See fmtgen_t3 in csrc/gen/fmtgen.cpp for the shape and why ranges are local edits."""
    ops = np.zeros(n_ops, dtype=MT_OP_DTYPE)
    segs = np.zeros(n_segments, dtype=SNAPSHOT_SEG_DTYPE)
    text = np.zeros(n_segments * 8 + n_ops * 3 + 1, dtype="<u2")
    n_text = _lib().fmtgen_t3(n_segments, n_ops, n_clients, max_lag, max_range, seed, 0, _p(segs), _p(text), _p(ops))
    if n_text < 0:
        raise ValueError(f"fmtgen_t3 failed ({n_text})")
    snaps = np.zeros(1, dtype=SNAPSHOT_DOC_DTYPE)
    snaps["first_seg"], snaps["n_header"], snaps["n_body"], snaps["loaded"] = 0, n_segments, 0, 1
    n_props = len(CLIENT_NAMES)
    return MergeTreeBatch(
        ops=ops,
        doc_op_offsets=np.array([0, n_ops], dtype=np.uint64),
        text=text[: max(1, n_text)].copy(),
        doc_init=np.zeros((1, 2), dtype=np.uint32),
        props_off=np.arange(n_props + 1, dtype=np.uint32),
        props_kv=np.array([(0 << 16) | (i + 1) for i in range(n_props)], dtype=np.uint32),
        keys=["client"],
        values=["null"] + [js_json(c) for c in CLIENT_NAMES],
        snapshots=snaps,
        snapshot_segs=segs,
    )


def as_legacy_load(batch: MergeTreeBatch, header_chars: int = 10000, props_every: int = 0) -> MergeTreeBatch:
    """A copy of a one-document summary-loaded batch (t3_stream) whose summary has the shape
    SnapshotLegacy.emit writes (snapshotlegacy.ts:55, 126-193; summary.py legacy_summary): a header
    chunk of the first segments up to header_chars UTF-16 units, the rest in the body chunk (loaded
    by loadBody's appends, snapshotLoader.ts:277-309). props_every > 0: every props_every-th segment
    spec carries props {"client": <name>} (props op (k // props_every) % n)."""
    import dataclasses

    lens = (batch.snapshot_segs["len"] & ~np.uint32(MT_SEG_MARKER)).astype(np.int64)
    n = len(lens)
    n_header = min(n, int(np.searchsorted(np.cumsum(lens), header_chars)) + 1)  # while length < header_chars
    snaps = batch.snapshots.copy()
    snaps["n_header"], snaps["n_body"] = n_header, n - n_header
    segs = batch.snapshot_segs.copy()
    if props_every:
        k = np.arange(n)
        pick = (k % props_every) == 0
        segs["props"] = np.where(pick, (k // props_every) % (len(batch.props_off) - 1), segs["props"]).astype(np.uint32)
    return dataclasses.replace(batch, snapshots=snaps, snapshot_segs=segs)


def emptying_stream(n_segments: int = 3000, pairs: int = 600, seed: int = 1) -> MergeTreeBatch:
    """A summary-loaded document (n_segments segments, beyond the large tier) that one remove
    empties; then `pairs` insert/remove pairs, minSeq trailing by one, so zamboni scours every block
    and packParent leaves the root childless (zamboni.ts:83-139); a final insert then grows the
    document from its empty root again."""
    import dataclasses

    base = t3_stream(n_segments, 1, n_clients=2, max_lag=1, seed=seed)
    total = int((base.snapshot_segs["len"] & ~np.uint32(MT_SEG_MARKER)).sum())
    text = list(base.text.tolist())
    ab = len(text)
    text += [ord("a"), ord("b")]
    hello = len(text)
    text += [ord(c) for c in "hello"]
    ops = np.zeros(2 * pairs + 2, dtype=MT_OP_DTYPE)
    ops[0] = (1, 0, 0, 0, total, 0, 0, 1, MT_REMOVE, 0)
    seq = 2
    for i in range(pairs):
        ops[1 + 2 * i] = (seq, seq - 1, seq - 1, 0, 0, ab, 2, 2, MT_INSERT, 0)
        ops[2 + 2 * i] = (seq + 1, seq, seq, 0, 2, 0, 0, 3, MT_REMOVE, 0)
        seq += 2
    ops[-1] = (seq, seq - 1, seq - 1, 0, 0, hello, 5, 2, MT_INSERT, 0)
    return dataclasses.replace(base, ops=ops, doc_op_offsets=np.array([0, len(ops)], dtype=np.uint64),
                               text=np.asarray(text, dtype="<u2"))


def with_insert_props(batch: MergeTreeBatch, every: int = 3) -> MergeTreeBatch:
    """A copy of a conflict-farm batch where every `every`-th insert (by seq) carries a segment
    spec {text, props} (SharedString.insertText(pos, text, props), sharedString.ts:198-200): by
    turns the client's {"client"} set, a two-key {"color", "client"} set, or {"color": null} (an
    empty property set: null values are dropped, properties.ts:68-95)."""
    import dataclasses

    ops = batch.ops.copy()
    n = len(batch.props_off) - 1
    kc, vr = len(batch.keys), len(batch.values)
    kv, off = [int(x) for x in batch.props_kv], [int(x) for x in batch.props_off]
    for c in range(n):  # n + c: {"color": red|blue, "client": c}
        kv += [(kc << 16) | (vr + (c & 1)), int(batch.props_kv[off[c]])]
        off.append(len(kv))
    kv.append(kc << 16)  # 2n: {"color": null}
    off.append(len(kv))
    ins = (ops["type"] == MT_INSERT) & (ops["seq"] % every == 0)
    pick = (ops["seq"] // every + ops["client"].astype(np.int32)) % 3
    pid = np.where(pick == 0, ops["client"].astype(np.int32), np.where(pick == 1, n + ops["client"].astype(np.int32), 2 * n))
    ops["pos2"] = np.where(ins, pid + 1, ops["pos2"])
    return dataclasses.replace(batch, ops=ops, props_off=np.asarray(off, np.uint32), props_kv=np.asarray(kv, np.uint32),
                               keys=batch.keys + ["color"], values=batch.values + [js_json("red"), js_json("blue")])


def replicate_batches(batches, n_docs: int) -> MergeTreeBatch:
    """One batch of n_docs documents cycling over the single-document batches given (plain streams:
    no summaries, relative positions or merge info), every copy with its own text in the arena.

    Used for the obliterate workload: the reference's 30 obliterate conflict farms
    (merge-tree/src/test/results/*-conflict-farm-with-obliterate-2.3.0.json, committed as
    tests/golden/replay_obliterate_2.3.0.npz) laid out as a batch of T1's size. Keys, values and
    props ops of the sources are merged; annotate payloads, insert props (pos2 - 1) and text offsets
    are rebased per copy.
    """
    keys, values = [], ["null"]
    kid, vid = {}, {"null": 0}
    kv_parts, off_parts, props_base = [], [], []
    n_props = 0
    for b in batches:
        if b.snapshots is not None or b.relpos is not None or b.snapshot_info is not None:
            raise ValueError("replicate_batches takes plain streams")
        if len(b.doc_op_offsets) != 2:
            raise ValueError("replicate_batches takes single-document batches")
        for k in b.keys:
            if k not in kid:
                kid[k] = len(keys)
                keys.append(k)
        kmap = np.array([kid[k] for k in b.keys] or [0], dtype=np.uint32)
        vmap = np.zeros(max(len(b.values), 1), dtype=np.uint32)
        for i, v in enumerate(b.values):
            if v not in vid:
                vid[v] = len(values)
                values.append(v)
            vmap[i] = vid[v]
        kv = b.props_kv.astype(np.uint32)
        kv_parts.append((kmap[kv >> 16] << 16) | vmap[kv & 0xFFFF])
        off_parts.append(b.props_off[1:].astype(np.uint64) + sum(len(p) for p in kv_parts[:-1]))
        props_base.append(n_props)
        n_props += len(b.props_off) - 1
    props_off = np.concatenate([np.zeros(1, dtype=np.uint64)] + off_parts).astype(np.uint32)
    props_kv = np.concatenate(kv_parts) if kv_parts else np.zeros(0, dtype=np.uint32)

    src = [i % len(batches) for i in range(n_docs)]
    n_ops = sum(len(batches[s].ops) for s in src)
    n_text = sum(len(batches[s].text) for s in src)
    if n_text >= 1 << 32:
        raise ValueError("text arena beyond 32-bit offsets")
    ops = np.empty(n_ops, dtype=MT_OP_DTYPE)
    text = np.empty(max(n_text, 1), dtype="<u2")
    offs = np.zeros(n_docs + 1, dtype=np.uint64)
    doc_init = np.zeros((n_docs, 2), dtype=np.uint32)
    # per source: which ops take a text offset / a props id
    shapes = []
    for s, b in enumerate(batches):
        t = b.ops["type"]
        ins = t == MT_INSERT
        shapes.append((ins, t == MT_ANNOTATE, ins & (b.ops["pos2"] > 0)))
    o = tx = 0
    for d, s in enumerate(src):
        b = batches[s]
        ins, ann, iprops = shapes[s]
        k = len(b.ops)
        blk = ops[o : o + k]
        blk[:] = b.ops
        blk["payload"][ins] += np.uint32(tx)
        blk["payload"][ann] += np.uint32(props_base[s])
        blk["pos2"][iprops] += np.int32(props_base[s])
        text[tx : tx + len(b.text)] = b.text
        doc_init[d] = (int(b.doc_init[0][0]) + tx, int(b.doc_init[0][1]))
        o += k
        tx += len(b.text)
        offs[d + 1] = o
    return MergeTreeBatch(ops=ops, doc_op_offsets=offs, text=text, doc_init=doc_init, props_off=props_off,
                          props_kv=props_kv, keys=keys, values=values)
