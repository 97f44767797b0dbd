"""ctypes binding of the parity oracle (oracle/_build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker or the CPU baseline — never as the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborc.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.orc_mt_new.restype = P
        L.orc_mt_free.argtypes = [P]
        L.orc_mt_insert_local.argtypes = [P, ctypes.c_int, P, ctypes.c_int]
        L.orc_mt_annotate_local.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.orc_mt_remove_local.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.orc_mt_start_collab.argtypes = [P, ctypes.c_int]
        L.orc_mt_apply_ops.argtypes = [P, P, ctypes.c_uint64, P, P, P]
        L.orc_mt_set_adjusts.argtypes = [P, P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.orc_mt_set_adjusts.restype = None
        L.orc_mt_set_relpos.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_mt_set_relpos.restype = None
        L.orc_mt_marker_present.argtypes = [P, ctypes.c_uint32]
        L.orc_mt_text.argtypes = [P, P, ctypes.c_int]
        L.orc_mt_dump.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.orc_mt_summary.argtypes = [P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P,
                                     ctypes.c_int, P, P]
        L.orc_mt_removers.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32]
        L.orc_mt_replay_batch.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, P, P,
                                          ctypes.c_uint32, P, ctypes.c_uint32, P, ctypes.c_uint32, P,
                                          ctypes.c_uint32, P, P, ctypes.c_uint32, P]
        L.orc_mt_replay_summary.argtypes = [P, ctypes.c_uint32, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P,
                                            ctypes.c_int, P, P]
        L.orc_mt_replay_timed.argtypes = [P, ctypes.c_uint32, ctypes.c_uint64, P, P, P, P, P, ctypes.c_uint32, P,
                                          ctypes.c_uint32, P, ctypes.c_uint32]
        L.orc_set_index.argtypes = [ctypes.c_int]
        L.orc_mt_replay_full.argtypes = [P, ctypes.c_uint32, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, P, P, P]
        L.orc_mt_full_take.argtypes = [P, P]
        L.orc_mt_replay_digest.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, P, P, P]
        L.orc_state_digest.argtypes = [P, P, P, P]
        L.orc_state_digest.restype = ctypes.c_uint64
        L.orc_map_replay.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, P, ctypes.c_uint32, P]
        L.orc_map_replay_sparse.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, P, P, ctypes.c_uint32, P]
        L.orc_map_summary.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, P,
                                      ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P]
        L.orc_xsadd_uint32.argtypes = [P, ctypes.c_int, P, ctypes.c_int]
        L.orc_xsadd_mixed.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int]
        L.orc_mt_local_length.argtypes = [P]
        L.orc_mt_pending_groups.argtypes = [P]
        L.orc_mt_regen_take.argtypes = [P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P]
        L.orc_mt_replay_regen.argtypes = [P, ctypes.c_uint32, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P]
        L.orc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _cstrs(strings):
    arr = (ctypes.c_char_p * max(1, len(strings)))()
    for i, s in enumerate(strings):
        arr[i] = s.encode("utf-8")
    return arr


class OracleError(RuntimeError):
    pass


class MergeTreeDoc:
    """One observer merge-tree (or a detached local string)."""

    def __init__(self):
        self.h = lib().orc_mt_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_mt_free(self.h)
            self.h = None

    def _check(self, rc):
        if rc != 0:
            raise OracleError(lib().orc_last_error().decode())

    def insert_local(self, pos: int, text: str):
        u = np.frombuffer(text.encode("utf-16-le", "surrogatepass"), dtype="<u2").copy()
        self._check(lib().orc_mt_insert_local(self.h, pos, _ptr(u), len(u)))

    def annotate_local(self, start: int, end: int, kv: list[int]):
        a = np.asarray(kv, dtype=np.uint32)
        self._check(lib().orc_mt_annotate_local(self.h, start, end, _ptr(a), len(a)))

    def remove_local(self, start: int, end: int):
        self._check(lib().orc_mt_remove_local(self.h, start, end))

    def start_collab(self, client: int = 0):
        lib().orc_mt_start_collab(self.h, client)

    def apply(self, ops: np.ndarray, arena: np.ndarray, props_off: np.ndarray, props_kv: np.ndarray):
        ops = np.ascontiguousarray(ops)
        self._check(lib().orc_mt_apply_ops(self.h, _ptr(ops), len(ops), _ptr(arena), _ptr(props_off),
                                           _ptr(props_kv)))

    def set_adjusts(self, adjusts: np.ndarray, value_num: np.ndarray):
        """Annotate-adjust rows (ADJUST_DTYPE) and per value id its number (NaN: none) for the ops
        applied next; the arrays must outlive those calls (kept here)."""
        self._adj = (np.ascontiguousarray(adjusts), np.ascontiguousarray(value_num, dtype=np.float64))
        lib().orc_mt_set_adjusts(self.h, _ptr(self._adj[0]), len(self._adj[0]), _ptr(self._adj[1]), len(self._adj[1]))

    def set_relpos(self, relpos: np.ndarray, marker_id_key: int):
        """The relpos table (RELPOS_DTYPE) and "markerId" key id for the ops applied next (kept here)."""
        self._rel = np.ascontiguousarray(relpos)
        lib().orc_mt_set_relpos(self.h, _ptr(self._rel), len(self._rel), marker_id_key)

    def marker_present(self, marker_value_id: int) -> bool:
        """A marker with that markerId value is in the document and not removed (locally or not)."""
        return bool(lib().orc_mt_marker_present(self.h, marker_value_id))

    def local_length(self) -> int:
        """getLength() from the local perspective (client.ts:1696)."""
        return int(lib().orc_mt_local_length(self.h))

    def pending_groups(self) -> int:
        return int(lib().orc_mt_pending_groups(self.h))

    def regen_take(self):
        """The ops REGEN events produced since the last call: (MT_OP_DTYPE records, their text)."""
        from fluidframework_amd.streams import MT_OP_DTYPE
        n, nt = ctypes.c_uint32(0), ctypes.c_uint32(0)
        lib().orc_mt_regen_take(self.h, None, 0, None, 0, ctypes.byref(n), ctypes.byref(nt))
        ops = np.zeros(max(1, n.value), dtype=MT_OP_DTYPE)
        text = np.zeros(max(1, nt.value), dtype="<u2")
        lib().orc_mt_regen_take(self.h, _ptr(ops), n.value, _ptr(text), nt.value, ctypes.byref(n), ctypes.byref(nt))
        return ops[: n.value], text[: nt.value]

    def text(self) -> str:
        n = lib().orc_mt_text(self.h, None, 0)
        buf = np.zeros(max(n, 1), dtype="<u2")
        lib().orc_mt_text(self.h, _ptr(buf), n)
        return buf[:n].tobytes().decode("utf-16-le", "surrogatepass")

    def dump(self, cap_leaves=1 << 16, cap_chars=1 << 20, cap_props=1024):
        from fluidframework_amd.native import DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE

        hdr = np.zeros(1, dtype=DOC_RESULT_DTYPE)
        leaves = np.zeros(cap_leaves, dtype=LEAF_DTYPE)
        chars = np.zeros(cap_chars, dtype="<u2")
        props = np.zeros(cap_props, dtype=PROPSET_DTYPE)
        lib().orc_mt_dump(self.h, _ptr(hdr), _ptr(leaves), cap_leaves, _ptr(chars), cap_chars,
                          _ptr(props), cap_props)
        h = hdr[0]
        return h, leaves[: h["n_leaves"]], chars[: h["n_chars"]], props[: h["n_props"]]

    def summary(self, keys: list[str], values: list[str], chunk_size: int = 10000):
        k, v = _cstrs(keys), _cstrs(values)
        hl, bl = ctypes.c_int(0), ctypes.c_int(0)
        n = lib().orc_mt_summary(self.h, k, len(keys), v, len(values), chunk_size, None, 0,
                                 ctypes.byref(hl), ctypes.byref(bl))
        buf = ctypes.create_string_buffer(n + 1)
        lib().orc_mt_summary(self.h, k, len(keys), v, len(values), chunk_size, buf, n,
                             ctypes.byref(hl), ctypes.byref(bl))
        raw = buf.raw[:n]
        header = raw[: hl.value].decode("utf-8")
        body = raw[hl.value : hl.value + bl.value].decode("utf-8") if bl.value else None
        return header, body


def mt_replay_regen(batch, doc: int):
    """f4: document `doc` replayed; (status, regenerated ops (MT_OP_DTYPE), their text) — the layout of
    fmt_mt_fetch_regen."""
    from fluidframework_amd.native import batch_struct
    from fluidframework_amd.streams import MT_OP_DTYPE
    b, keep = batch_struct(batch)
    n, nt = ctypes.c_uint32(0), ctypes.c_uint32(0)
    lib().orc_mt_replay_regen(ctypes.byref(b), doc, None, 0, None, 0, ctypes.byref(n), ctypes.byref(nt))
    ops = np.zeros(max(1, n.value), dtype=MT_OP_DTYPE)
    text = np.zeros(max(1, nt.value), dtype="<u2")
    rc = lib().orc_mt_replay_regen(ctypes.byref(b), doc, _ptr(ops), n.value, _ptr(text), nt.value,
                                   ctypes.byref(n), ctypes.byref(nt))
    del keep
    return rc, ops[: n.value], text[: nt.value]


def mt_replay_batch(batch, doc_begin=0, doc_end=None, threads=1, cap_leaves=4096, cap_chars=1 << 16,
                    cap_props=64, outputs=True, cap_catchup=0, numbers=None):
    """Replay a MergeTreeBatch; returns (rc, headers, leaves, chars, props, seconds).

    With cap_catchup > 0 the catch-up ranges of FMT_MT_F_CATCHUP ops are recorded too and returned
    as a 7th element, shape (n_docs, cap_catchup) of CATCHUP_DTYPE (headers' n_catchup counts them).
    With a list `numbers`, each document's computed annotate-adjust numbers (value ids
    FMT_MT_VALUE_COMPUTED + index) are appended to it as a float64 array.
    """
    from fluidframework_amd.native import (CATCHUP_DTYPE, DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE,
                                           batch_struct)

    doc_end = batch.n_docs if doc_end is None else doc_end
    n = doc_end - doc_begin
    hdrs = np.zeros(n, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(n * cap_leaves, dtype=LEAF_DTYPE) if outputs else None
    chars = np.zeros(n * cap_chars, dtype="<u2") if outputs else None
    props = np.zeros(n * cap_props, dtype=PROPSET_DTYPE) if outputs else None
    catchup = np.zeros(n * cap_catchup, dtype=CATCHUP_DTYPE) if cap_catchup else None
    secs = ctypes.c_double(0)
    cap_nums = 4096 if numbers is not None else 0
    nums = np.zeros(n * cap_nums, dtype=np.float64) if cap_nums else None
    n_nums = np.zeros(n, dtype=np.uint32) if cap_nums else None
    b, keep = batch_struct(batch)
    rc = lib().orc_mt_replay_batch(ctypes.byref(b), doc_begin, doc_end, threads, _ptr(hdrs),
                                   _ptr(leaves), cap_leaves, _ptr(chars), cap_chars, _ptr(props),
                                   cap_props, _ptr(catchup), cap_catchup, ctypes.byref(secs),
                                   _ptr(nums), cap_nums, _ptr(n_nums))
    del keep
    if numbers is not None:
        for i in range(n):
            numbers.append(nums[i * cap_nums: i * cap_nums + min(int(n_nums[i]), cap_nums)].copy())
    if outputs:
        leaves = leaves.reshape(n, cap_leaves)
        chars = chars.reshape(n, cap_chars)
        props = props.reshape(n, cap_props)
    if cap_catchup:
        return rc, hdrs, leaves, chars, props, secs.value, catchup.reshape(n, cap_catchup)
    return rc, hdrs, leaves, chars, props, secs.value


def mt_replay_digest(batch, doc_begin=0, doc_end=None, threads=1):
    """Replay documents [doc_begin, doc_end) and return (rc, digests uint64[n], statuses int32[n],
    replay seconds): each document's state digest (what fmt_mt_state_digest computes on
    the device); the seconds time the replays alone, the digests are taken afterwards."""
    from fluidframework_amd.native import batch_struct

    doc_end = batch.n_docs if doc_end is None else doc_end
    n = doc_end - doc_begin
    dig = np.zeros(max(n, 1), dtype=np.uint64)
    st = np.zeros(max(n, 1), dtype=np.int32)
    secs = ctypes.c_double(0)
    b, keep = batch_struct(batch)
    rc = lib().orc_mt_replay_digest(ctypes.byref(b), doc_begin, doc_end, threads, _ptr(dig), _ptr(st), ctypes.byref(secs))
    del keep
    return rc, dig[:n], st[:n], secs.value


def state_digest(hdr, leaves, chars, props) -> int:
    """The state digest of one dumped document (the oracle's restatement of the definition)."""
    from fluidframework_amd.native import DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE

    h = np.ascontiguousarray(np.asarray(hdr).reshape(1), dtype=DOC_RESULT_DTYPE)
    lv = np.ascontiguousarray(leaves, dtype=LEAF_DTYPE) if len(leaves) else np.zeros(1, LEAF_DTYPE)
    ch = np.ascontiguousarray(chars, dtype="<u2") if len(chars) else np.zeros(1, "<u2")
    pr = np.ascontiguousarray(props, dtype=PROPSET_DTYPE) if len(props) else np.zeros(1, PROPSET_DTYPE)
    return int(lib().orc_state_digest(_ptr(h), _ptr(lv), _ptr(ch), _ptr(pr)))


def mt_replay_summary(batch, doc: int, keys, values, chunk_size: int = 10000):
    """Document `doc` of a batch replayed by the oracle, then its legacy summary (header, body) from
    the oracle's own SnapshotLegacy restatement; raises on a replay failure."""
    from fluidframework_amd.native import batch_struct

    kk, vv = _cstrs(keys), _cstrs(values)
    b, keep = batch_struct(batch)
    hl, bl = ctypes.c_int(0), ctypes.c_int(0)
    n = lib().orc_mt_replay_summary(ctypes.byref(b), doc, kk, len(keys), vv, len(values), chunk_size, None, 0,
                                    ctypes.byref(hl), ctypes.byref(bl))
    if n < 0:
        raise RuntimeError(f"oracle replay failed ({n}): {lib().orc_last_error().decode()}")
    buf = ctypes.create_string_buffer(n)
    lib().orc_mt_replay_summary(ctypes.byref(b), doc, kk, len(keys), vv, len(values), chunk_size, buf, n,
                                ctypes.byref(hl), ctypes.byref(bl))
    del keep
    raw = buf.raw[:n]
    return raw[: hl.value].decode("utf-8"), (raw[hl.value:].decode("utf-8") if bl.value else None)


def mt_replay_full(batch, doc: int, keys, values, chunk_size: int = 10000):
    """Document `doc` replayed ONCE by the oracle: (state digest, legacy header, body or None, catch-up
    ranges of its FMT_MT_F_CATCHUP ops, final minSeq is in the digest's header). Raises on failure."""
    from fluidframework_amd.native import CATCHUP_DTYPE, batch_struct

    kk, vv = _cstrs(keys), _cstrs(values)
    b, keep = batch_struct(batch)
    dig = ctypes.c_uint64(0)
    hl, bl, ncu = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_uint32(0)
    rc = lib().orc_mt_replay_full(ctypes.byref(b), doc, kk, len(keys), vv, len(values), chunk_size, ctypes.byref(dig),
                                  ctypes.byref(hl), ctypes.byref(bl), ctypes.byref(ncu))
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle replay failed ({rc}): {lib().orc_last_error().decode()}")
    buf = ctypes.create_string_buffer(hl.value + bl.value + 1)
    cu = np.zeros(max(ncu.value, 1), dtype=CATCHUP_DTYPE)
    lib().orc_mt_full_take(buf, _ptr(cu))
    raw = buf.raw[: hl.value + bl.value]
    return (int(dig.value), raw[: hl.value].decode("utf-8"), raw[hl.value:].decode("utf-8") if bl.value else None,
            cu[: ncu.value])


def set_index(on: bool):
    """Replays use the per-block remote-length index (MergeTree::enableIndex): same results, O(log)
    block lengths instead of subtree sums (what makes a 10M-segment T3 document replayable)."""
    lib().orc_set_index(1 if on else 0)


def mt_replay_timed(batch, doc=0, max_ops=0, cap_leaves=0, cap_chars=0, cap_props=64):
    """Replay one document (its first max_ops ops; all with 0), timing load and ops separately.
    Returns (rc, header, leaves, chars, props, load_s, ops_s, ops_done)."""
    from fluidframework_amd.native import DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE, batch_struct

    hdr = np.zeros(1, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(max(cap_leaves, 1), dtype=LEAF_DTYPE)
    chars = np.zeros(max(cap_chars, 1), dtype="<u2")
    props = np.zeros(max(cap_props, 1), dtype=PROPSET_DTYPE)
    ls, os_, nd = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_uint64(0)
    b, keep = batch_struct(batch)
    rc = lib().orc_mt_replay_timed(ctypes.byref(b), doc, max_ops, ctypes.byref(ls), ctypes.byref(os_), ctypes.byref(nd),
                                   _ptr(hdr), _ptr(leaves), cap_leaves, _ptr(chars), cap_chars, _ptr(props), cap_props)
    del keep
    return rc, hdr[0], leaves[:cap_leaves], chars[:cap_chars], props, ls.value, os_.value, nd.value


def map_replay(batch, threads=1):
    """Replay a MapBatch; returns (slots[n_docs, key_bound], seconds)."""
    from fluidframework_amd.native import MAP_SLOT_DTYPE

    out = np.zeros(batch.n_docs * batch.key_bound, dtype=MAP_SLOT_DTYPE)
    secs = ctypes.c_double(0)
    ops = np.ascontiguousarray(batch.ops)
    offs = np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64)
    rc = lib().orc_map_replay(_ptr(ops), _ptr(offs), batch.n_docs, batch.key_bound, _ptr(out), threads,
                              ctypes.byref(secs))
    if rc != 0:
        raise OracleError("map replay failed")
    return out.reshape(batch.n_docs, batch.key_bound), secs.value


def map_replay_sparse(batch, threads=1):
    """Replay a MapBatch keeping only live entries (any key pool): returns (counts[n_docs], entries
    packed in document order, each document's in Map order, seconds) — the sparse path's layout."""
    from fluidframework_amd.native import MAP_ENTRY_DTYPE

    counts = np.zeros(batch.n_docs, dtype=np.uint32)
    ent = np.zeros(max(len(batch.ops), 1), dtype=MAP_ENTRY_DTYPE)
    secs = ctypes.c_double(0)
    ops = np.ascontiguousarray(batch.ops)
    offs = np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64)
    rc = lib().orc_map_replay_sparse(_ptr(ops), _ptr(offs), batch.n_docs, batch.key_bound, _ptr(counts), _ptr(ent),
                                     threads, ctypes.byref(secs))
    if rc != 0:
        raise OracleError("map replay failed")
    c = counts.astype(np.int64)
    first = np.cumsum(c) - c  # packed index of each document's first entry
    take = np.arange(int(c.sum()), dtype=np.int64) + np.repeat(offs[:-1].astype(np.int64) - first, c)
    return counts, ent[take], secs.value


def map_pending(batch):
    """The local client's optimistic view of every document (MapKernel pendingData over the sequenced
    entries, oracle/map.cpp PendingMap): (counts[n_docs], status[n_docs], entries packed in document
    order) — the layout of fmt_map_pending_fetch."""
    from fluidframework_amd.native import MAP_ENTRY_DTYPE

    ops = np.ascontiguousarray(batch.ops)
    offs = np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64)
    ev = np.ascontiguousarray(batch.local_ops)
    eo = np.ascontiguousarray(batch.local_offsets, dtype=np.uint64)
    counts = np.zeros(batch.n_docs, dtype=np.uint32)
    status = np.zeros(batch.n_docs, dtype=np.int32)
    ent = np.zeros(max(len(ops) + len(ev), 1), dtype=MAP_ENTRY_DTYPE)
    lib().orc_map_pending(_ptr(ops), _ptr(offs), ctypes.c_uint32(batch.n_docs), ctypes.c_uint32(batch.key_bound),
                          _ptr(ev), _ptr(eo), _ptr(counts), _ptr(status), _ptr(ent))
    c = counts.astype(np.int64)
    first = np.cumsum(c) - c
    base = offs[:-1].astype(np.int64) + eo[:-1].astype(np.int64)
    take = np.arange(int(c.sum()), dtype=np.int64) + np.repeat(base - first, c)
    return counts, status, ent[take]


def map_summary(batch, doc: int):
    ops = np.ascontiguousarray(batch.ops)
    b, e = int(batch.doc_op_offsets[doc]), int(batch.doc_op_offsets[doc + 1])
    k, v = _cstrs(batch.keys), _cstrs(batch.values)
    nb = ctypes.c_int(0)
    n = lib().orc_map_summary(_ptr(ops), b, e, batch.key_bound, k, len(batch.keys), v, len(batch.values),
                              None, 0, ctypes.byref(nb))
    buf = ctypes.create_string_buffer(n + 1)
    lib().orc_map_summary(_ptr(ops), b, e, batch.key_bound, k, len(batch.keys), v, len(batch.values),
                          buf, n, ctypes.byref(nb))
    parts = buf.raw[:n].split(b"\0")
    return parts[0].decode(), [p.decode() for p in parts[1 : 1 + nb.value]]


def xsadd_uint32(seed, n):
    s = np.asarray(seed, dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    lib().orc_xsadd_uint32(_ptr(s), len(s), _ptr(out), n)
    return out


def xsadd_mixed(seed, kinds):
    s = np.asarray(seed, dtype=np.uint32)
    k = np.asarray(kinds, dtype=np.int32)
    out = np.zeros(len(k), dtype=np.float64)
    lib().orc_xsadd_mixed(_ptr(s), len(s), _ptr(k), _ptr(out), len(k))
    return out


def mt_removers(batch, doc: int, cap: int = 1 << 16):
    """Every remove stamp of every final leaf of `doc`, in stamp order:
    {leaf index: [(client, seq, kind), ...]} with kind 0 = setRemove, 1 = sliceRemove (obliterate)."""
    from fluidframework_amd.native import batch_struct

    out = np.zeros(4 * cap, dtype=np.int32)
    b, keep = batch_struct(batch)
    n = lib().orc_mt_removers(ctypes.byref(b), doc, _ptr(out), cap)
    del keep
    if n < 0:
        raise OracleError(f"remove-order replay failed ({n})")
    res = {}
    for k in range(min(n, cap)):
        q = out[4 * k : 4 * k + 4]
        res.setdefault(int(q[0]), []).append((int(q[1]), int(q[2]), int(q[3])))
    return res


def js_map_replay(batch, workers, tmpdir=None, reps=1):
    """The JS restatement of the SharedMap observer path (oracle/js/map_observer.js) on `workers`
    worker_threads: returns (per-document entry hashes, its JSON stats line). CPU baseline only."""
    import json
    import shutil
    import subprocess
    import tempfile

    node = shutil.which("node")
    if node is None:
        raise OracleError("node is not on PATH")
    d = tempfile.mkdtemp(dir=tmpdir)
    try:
        ops = os.path.join(d, "ops.bin")
        offs = os.path.join(d, "offs.bin")
        keys = os.path.join(d, "keys.json")
        out = os.path.join(d, "hashes.bin")
        np.ascontiguousarray(batch.ops).tofile(ops)
        np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64).tofile(offs)
        names = list(batch.keys) + [str(k) for k in range(len(batch.keys), batch.key_bound)]
        with open(keys, "w") as f:
            json.dump(names, f)
        script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "js", "map_observer.js")
        r = subprocess.run([node, script, ops, offs, keys, str(workers), out, str(reps)], capture_output=True, text=True)
        if r.returncode != 0:
            raise OracleError(f"map_observer.js failed: {r.stderr[-2000:]}")
        return np.fromfile(out, dtype=np.uint32), json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        shutil.rmtree(d, ignore_errors=True)


def map_entry_hashes(slots):
    """Per-document hash of the live entries in Map iteration order (birth seq), as map_observer.js
    folds them: FNV-1a-style over (key id, value id)."""
    slots = np.asarray(slots)
    out = np.zeros(len(slots), dtype=np.uint32)
    for d in range(len(slots)):
        live = np.nonzero(slots[d]["value"] != 0xFFFFFFFF)[0]
        h = 0x811C9DC5
        for k in live[np.argsort(slots[d]["birth_seq"][live], kind="stable")]:
            h = ((h ^ int(k)) * 16777619) & 0xFFFFFFFF
            h = ((h ^ int(slots[d]["value"][k])) * 16777619) & 0xFFFFFFFF
        out[d] = h
    return out


def js_mt_replay(batch, workers, tmpdir=None, reps=1):
    """The JS restatement of the SharedString observer path (oracle/js/mt_observer.js) on `workers`
    worker_threads: returns (per-document FNV-1a hashes of the final text, its JSON stats line).
    CPU baseline only."""
    import json
    import shutil
    import subprocess
    import tempfile

    node = shutil.which("node")
    if node is None:
        raise OracleError("node is not on PATH")
    d = tempfile.mkdtemp(dir=tmpdir)
    try:
        n = batch.n_docs
        np.ascontiguousarray(batch.ops).tofile(os.path.join(d, "ops.bin"))
        np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64).tofile(os.path.join(d, "offs.bin"))
        np.ascontiguousarray(batch.text, dtype="<u2").tofile(os.path.join(d, "text.bin"))
        init = batch.doc_init if batch.doc_init is not None else np.zeros((n, 2), dtype=np.uint32)
        np.ascontiguousarray(init, dtype=np.uint32).tofile(os.path.join(d, "init.bin"))
        np.ascontiguousarray(batch.props_off, dtype=np.uint32).tofile(os.path.join(d, "props_off.bin"))
        np.ascontiguousarray(batch.props_kv, dtype=np.uint32).tofile(os.path.join(d, "props_kv.bin"))
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump({"keys": list(batch.keys), "values": list(batch.values)}, f)
        script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "js", "mt_observer.js")
        r = subprocess.run([node, script, d, str(workers), str(reps)], capture_output=True, text=True)
        if r.returncode != 0:
            raise OracleError(f"mt_observer.js failed: {r.stderr[-2000:]}")
        return np.fromfile(os.path.join(d, "hashes.bin"), dtype=np.uint32)[:n], json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        shutil.rmtree(d, ignore_errors=True)


def text_hash(units) -> int:
    """FNV-1a over UTF-16 code units, as mt_observer.js folds a document's final text."""
    h = 0x811C9DC5
    for u in np.asarray(units, dtype=np.uint16).tolist():
        h = ((h ^ u) * 16777619) & 0xFFFFFFFF
    return h


def visible_units(hdr, leaves, chars):
    """The UTF-16 units of a replayed document's visible text (oracle outputs)."""
    parts = [chars[int(L["char_off"]): int(L["char_off"]) + int(L["len"])] for L in leaves[: int(hdr["n_leaves"])]
             if int(L["rm_seq"]) == 0x7FFFFFFF and not int(L["pad"]) & 0x8000]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint16)
