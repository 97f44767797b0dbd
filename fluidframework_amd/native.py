"""ctypes binding of libfmt.so (include/fmt.h), the HIP engine for gfx950.

There is no CPU fallback: if the library or a gfx950 device is missing, every call raises
`EngineUnavailable`. Result dtypes below mirror the C structs byte for byte.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfmt.so")

FMT_OK = 0
FMT_E_USAGE, FMT_E_DATA, FMT_E_CAPACITY, FMT_E_DEVICE, FMT_E_UNSUPPORTED = -1, -2, -3, -4, -5
STATUS_NAMES = {0: "OK", -1: "USAGE", -2: "DATA", -3: "CAPACITY", -4: "DEVICE", -5: "UNSUPPORTED"}

LEAF_DTYPE = np.dtype(
    [
        ("ins_seq", "<i4"),
        ("rm_seq", "<i4"),
        ("rm_clients", "<u8"),
        ("char_off", "<u4"),
        ("len", "<u4"),
        ("ins_client", "<i2"),
        ("props", "<u2"),
        ("block", "<u2"),
        ("pad", "<u2"),
    ]
)
assert LEAF_DTYPE.itemsize == 32

DOC_RESULT_DTYPE = np.dtype(
    [
        ("status", "<i4"),
        ("fail_seq", "<i4"),
        ("cur_seq", "<i4"),
        ("min_seq", "<i4"),
        ("n_leaves", "<u4"),
        ("n_chars", "<u4"),
        ("n_props", "<u4"),
        ("n_blocks", "<u4"),
        ("depth", "<u4"),
        ("visible_len", "<u4"),
        ("n_catchup", "<u4"),
        ("n_rm_order", "<u4"),
    ]
)
assert DOC_RESULT_DTYPE.itemsize == 48

# fmt_mt_remove_order: a later remove stamp of a leaf (leaf index, client, seq, kind 0 = setRemove /
# 1 = sliceRemove); FMT_MT_LEAF_GONE leaf
RM_ORDER_DTYPE = np.dtype([("leaf", "<u4"), ("client", "<i4"), ("seq", "<i4"), ("kind", "<u4")])
LEAF_GONE = 0xFFFFFFFF

CATCHUP_DTYPE = np.dtype([("op", "<u4"), ("pos1", "<i4"), ("pos2", "<i4"), ("type", "<u4")])

from .streams import (NO_MARKER, RELPOS_DTYPE, SNAPSHOT_DOC_DTYPE, SNAPSHOT_INFO_DTYPE, SNAPSHOT_SEG_DTYPE,  # noqa: E402
                      STAMP_DTYPE)  # (include/fmt.h layouts)

PROPS_MAX = 8        # fmt.h FMT_MT_PROPS_MAX: entries per prop-set record
PROPS_KEYS_MAX = 128  # fmt.h FMT_MT_PROPS_KEYS_MAX: entries per prop set
PROPS_CONT = 0xFFFFFFFF  # fmt.h FMT_MT_PROPS_CONT: n of a continuation record
MAP_PENDING_MAX_EVENTS = 16384  # fmt.h FMT_MAP_PENDING_MAX_EVENTS: local events per document
PROPSET_DTYPE = np.dtype([("n", "<u4"), ("kv", "<u4", (PROPS_MAX,))])


def propset_entries(table, pid: int) -> tuple:
    """The (key << 16 | value) entries of the prop set whose first record is table[pid]; a set wider
    than PROPS_MAX continues in the following records (fmt.h fmt_mt_propset)."""
    n = int(table[pid]["n"])
    if n <= PROPS_MAX:
        return tuple(int(x) for x in table[pid]["kv"][:n])
    rec = table[pid : pid + (n + PROPS_MAX - 1) // PROPS_MAX]["kv"].reshape(-1)
    return tuple(int(x) for x in rec[:n])
assert PROPSET_DTYPE.itemsize == 36

MAP_SLOT_DTYPE = np.dtype([("value", "<u4"), ("birth_seq", "<u4")])
MAP_ENTRY_DTYPE = np.dtype([("key", "<u4"), ("value", "<u4"), ("birth_seq", "<u4")])  # fmt_map_entry


class FmtMtBatch(ctypes.Structure):
    _fields_ = [
        ("ops", ctypes.c_void_p),
        ("n_ops", ctypes.c_uint64),
        ("doc_op_offsets", ctypes.c_void_p),
        ("n_docs", ctypes.c_uint32),
        ("text", ctypes.c_void_p),
        ("text_len", ctypes.c_uint64),
        ("doc_init", ctypes.c_void_p),
        ("props_off", ctypes.c_void_p),
        ("n_props_ops", ctypes.c_uint32),
        ("props_kv", ctypes.c_void_p),
        ("snapshots", ctypes.c_void_p),
        ("snapshot_segs", ctypes.c_void_p),
        ("n_snapshot_segs", ctypes.c_uint64),
        ("relpos", ctypes.c_void_p),
        ("n_relpos", ctypes.c_uint32),
        ("marker_id_key", ctypes.c_uint32),
        ("snapshot_info", ctypes.c_void_p),
        ("snapshot_stamps", ctypes.c_void_p),
        ("n_snapshot_stamps", ctypes.c_uint64),
        ("adjusts", ctypes.c_void_p),
        ("n_adjusts", ctypes.c_uint32),
        ("n_values", ctypes.c_uint32),
        ("value_num", ctypes.c_void_p),
        ("doc_value_base", ctypes.c_void_p),
    ]


from .streams import ADJUST_DTYPE  # noqa: E402  (include/fmt.h fmt_mt_adjust, 32 bytes)

assert ADJUST_DTYPE.itemsize == 32


class FmtStats(ctypes.Structure):
    _fields_ = [
        ("kernel_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("ops", ctypes.c_uint64),
        ("docs", ctypes.c_uint64),
        ("bytes_read", ctypes.c_uint64),
        ("bytes_written", ctypes.c_uint64),
        ("launches", ctypes.c_uint64),
    ]


class FmtConfig(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("stream", ctypes.c_void_p),
        ("reserved", ctypes.c_uint32 * 4),
    ]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def batch_struct(batch):
    """Build an fmt_mt_batch over a MergeTreeBatch's numpy arrays; returns (struct, keepalive)."""
    keep = [
        np.ascontiguousarray(batch.ops),
        np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64),
        np.ascontiguousarray(batch.text, dtype="<u2"),
        np.ascontiguousarray(batch.doc_init, dtype=np.uint32),
        np.ascontiguousarray(batch.props_off, dtype=np.uint32),
        np.ascontiguousarray(batch.props_kv, dtype=np.uint32) if len(batch.props_kv) else np.zeros(1, np.uint32),
    ]
    snaps = getattr(batch, "snapshots", None)
    segs = getattr(batch, "snapshot_segs", None)
    if snaps is not None:
        keep.append(np.ascontiguousarray(snaps, dtype=SNAPSHOT_DOC_DTYPE))
        keep.append(np.ascontiguousarray(segs, dtype=SNAPSHOT_SEG_DTYPE) if len(segs) else
                    np.zeros(1, dtype=SNAPSHOT_SEG_DTYPE))
    relpos = getattr(batch, "relpos", None)
    rel = np.ascontiguousarray(relpos, dtype=RELPOS_DTYPE) if relpos is not None and len(relpos) else None
    b = FmtMtBatch(
        _ptr(keep[0]), len(keep[0]), _ptr(keep[1]), len(keep[1]) - 1, _ptr(keep[2]), len(keep[2]),
        _ptr(keep[3]), _ptr(keep[4]), len(keep[4]) - 1, _ptr(keep[5]),
        _ptr(keep[6]) if snaps is not None else None, _ptr(keep[7]) if snaps is not None else None,
        len(segs) if snaps is not None else 0,
        _ptr(rel) if rel is not None else None, len(rel) if rel is not None else 0,
        int(getattr(batch, "marker_id_key", NO_MARKER)),
    )
    if rel is not None:
        keep.append(rel)
    info = getattr(batch, "snapshot_info", None)
    if snaps is not None and info is not None:
        inf = np.ascontiguousarray(info, dtype=SNAPSHOT_INFO_DTYPE)
        st = getattr(batch, "snapshot_stamps", None)
        stp = np.ascontiguousarray(st, dtype=STAMP_DTYPE) if st is not None and len(st) else np.zeros(1, STAMP_DTYPE)
        b.snapshot_info, b.snapshot_stamps = _ptr(inf), _ptr(stp)
        b.n_snapshot_stamps = 0 if st is None else len(st)
        keep += [inf, stp]
    adj = getattr(batch, "adjusts", None)
    if adj is not None and len(adj):
        a = np.ascontiguousarray(adj, dtype=ADJUST_DTYPE)
        vn = np.ascontiguousarray(batch.value_num, dtype=np.float64)
        b.adjusts, b.n_adjusts, b.value_num, b.n_values = _ptr(a), len(a), _ptr(vn), len(vn)
        keep += [a, vn]
    vb = getattr(batch, "value_base", None)
    if vb is not None:
        vba = np.ascontiguousarray(vb, dtype=np.uint32)
        b.doc_value_base = _ptr(vba)
        keep.append(vba)
    return b, keep


class EngineUnavailable(RuntimeError):
    """libfmt.so is missing or no gfx950 device is usable. There is deliberately no fallback."""


class FmtSummaryTiming(ctypes.Structure):  # fmt_summary_timing
    _fields_ = [("kernel_ms", ctypes.c_double), ("fetch_ms", ctypes.c_double), ("format_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("threads", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fmt error {STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_libs = {}


def lib(path: str | None = None) -> ctypes.CDLL:
    """The engine library (default: the in-tree libfmt.so; `path` selects an experimental build)."""
    path = path or LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise EngineUnavailable(f"{path} not built (run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.fmt_open.argtypes = [ctypes.POINTER(FmtConfig), ctypes.POINTER(P)]
        L.fmt_close.argtypes = [P]
        L.fmt_last_error.argtypes = [P]
        L.fmt_last_error.restype = ctypes.c_char_p
        L.fmt_sync.argtypes = [P]
        L.fmt_get_stats.argtypes = [P, ctypes.POINTER(FmtStats)]
        L.fmt_device_info.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
        L.fmt_map_load.argtypes = [P, P, U64, P, U32, U32]
        L.fmt_map_run.argtypes = [P]
        L.fmt_map_fetch.argtypes = [P, P]
        L.fmt_map_replay_device.argtypes = [P, P, P, U32, U32, P]
        L.fmt_map_check.argtypes = [P]
        L.fmt_map_load_sparse.argtypes = [P, P, U64, P, U32, U32]
        L.fmt_mt_summarize_legacy.argtypes = [P, P, U32, P, U32, U32, U32, ctypes.POINTER(FmtSummaryTiming)]
        L.fmt_mt_summary_blobs.argtypes = [P, U32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                           ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t)]
        L.fmt_map_run_sparse.argtypes = [P]
        L.fmt_map_fetch_sparse.argtypes = [P, P, P, U64, ctypes.POINTER(U64)]
        L.fmt_mt_load.argtypes = [P, ctypes.POINTER(FmtMtBatch)]
        L.fmt_mt_run.argtypes = [P]
        L.fmt_mt_fetch_headers.argtypes = [P, P]
        L.fmt_mt_fetch_doc.argtypes = [P, U32, P, U32, P, U32, P, U32]
        L.fmt_mt_fetch_catchup.argtypes = [P, U32, P, U32]
        L.fmt_mt_fetch_catchup_all.argtypes = [P, P, P, U64]
        L.fmt_mt_fetch_remove_order.argtypes = [P, U32, P, U32]
        L.fmt_mt_fetch_numbers.argtypes = [P, U32, P, U32, ctypes.POINTER(U32)]
        L.fmt_mt_capacity.argtypes = [ctypes.POINTER(U32)] * 3
        for name, args in (("fmt_mt_state_digest", [P, P]), ("fmt_mt_fetch_legacy_props", [P, U32, P, U32]),
                           ("fmt_mt_fetch_rm_clients_hi", [P, U32, P, U32]),
                           ("fmt_mt_fetch_rm_clients_hi2", [P, U32, P, U32]),
                           ("fmt_map_pending_run", [P, P, U64, P]),
                           ("fmt_mt_fetch_regen", [P, U32, P, U32, P, U32, ctypes.POINTER(U32), ctypes.POINTER(U32)]),
                           ("fmt_map_pending_fetch", [P, P, P, P, U64, ctypes.POINTER(U64)])):
            if path == LIB_PATH or hasattr(L, name):  # (older experimental builds may lack them)
                getattr(L, name).argtypes = args
        _libs[path] = L
    return _libs[path]


EXPORTED_SYMBOLS = [
    "fmt_open", "fmt_close", "fmt_last_error", "fmt_sync", "fmt_get_stats", "fmt_device_info",
    "fmt_map_load", "fmt_map_run", "fmt_map_fetch", "fmt_map_replay_device", "fmt_map_check",
    "fmt_map_load_sparse", "fmt_map_run_sparse", "fmt_map_fetch_sparse",
    "fmt_mt_summarize_legacy", "fmt_mt_summary_blobs",
    "fmt_mt_load", "fmt_mt_run", "fmt_mt_fetch_headers", "fmt_mt_fetch_doc", "fmt_mt_fetch_catchup",
    "fmt_mt_fetch_catchup_all", "fmt_mt_fetch_remove_order", "fmt_mt_fetch_numbers", "fmt_mt_capacity",
    "fmt_mt_state_digest", "fmt_mt_fetch_legacy_props", "fmt_map_pending_run", "fmt_map_pending_fetch",
    "fmt_mt_fetch_regen", "fmt_mt_fetch_rm_clients_hi", "fmt_mt_fetch_rm_clients_hi2",
]


def capacity():
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    lib().fmt_mt_capacity(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


class Engine:
    """One fmt_ctx bound to one HIP device (one per process/rank)."""

    def __init__(self, device: int = 0, stream: int | None = None, lib_path: str | None = None):
        self.L = L = lib(lib_path)
        cfg = FmtConfig(device, 0, stream, (ctypes.c_uint32 * 4)())
        h = ctypes.c_void_p()
        rc = L.fmt_open(ctypes.byref(cfg), ctypes.byref(h))
        if rc != FMT_OK:
            msg = L.fmt_last_error(h).decode() if h.value else "fmt_open failed"
            if h.value:
                L.fmt_close(h)
            raise EngineUnavailable(msg)
        self.h = h
        self._keep = None

    def close(self):
        if self.h:
            self.L.fmt_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != FMT_OK:
            raise EngineError(rc, self.L.fmt_last_error(self.h).decode())

    def sync(self):
        self._check(self.L.fmt_sync(self.h))

    def stats(self) -> FmtStats:
        s = FmtStats()
        self._check(self.L.fmt_get_stats(self.h, ctypes.byref(s)))
        return s

    def device_info(self) -> str:
        buf = ctypes.create_string_buffer(256)
        self.L.fmt_device_info(self.h, buf, 256)
        return buf.value.decode()

    # ---- SharedMap
    def map_load(self, batch):
        ops = np.ascontiguousarray(batch.ops)
        offs = np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64)
        self._check(self.L.fmt_map_load(self.h, _ptr(ops), len(ops), _ptr(offs), batch.n_docs, batch.key_bound))
        self._map_shape = (batch.n_docs, batch.key_bound)

    def map_run(self):
        self._check(self.L.fmt_map_run(self.h))

    def map_replay_device(self, d_ops: int, d_offsets: int, n_docs: int, key_bound: int, d_out: int):
        """fmt_map_replay_device on caller-owned device pointers (e.g. torch tensors' data_ptr())."""
        self._check(self.L.fmt_map_replay_device(self.h, d_ops, d_offsets, n_docs, key_bound, d_out))

    def map_check(self):
        """Raises EngineError(FMT_E_DATA) when the last map run saw a key id >= key_bound."""
        self._check(self.L.fmt_map_check(self.h))

    def map_fetch(self) -> np.ndarray:
        out = np.zeros(self._map_shape[0] * self._map_shape[1], dtype=MAP_SLOT_DTYPE)
        self._check(self.L.fmt_map_fetch(self.h, _ptr(out)))
        return out.reshape(self._map_shape)

    # sparse path (key pools of any size): one entry per live key, per document in birth order
    def map_load_sparse(self, batch):
        ops = np.ascontiguousarray(batch.ops)
        offs = np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64)
        self._check(self.L.fmt_map_load_sparse(self.h, _ptr(ops), len(ops), _ptr(offs), batch.n_docs, batch.key_bound))
        self._map_shape = (batch.n_docs, batch.key_bound)
        self._map_nops = len(ops)

    def map_run_sparse(self):
        self._check(self.L.fmt_map_run_sparse(self.h))

    def map_fetch_sparse(self):
        """(counts[n_docs], entries[sum(counts)]) with MAP_ENTRY_DTYPE, documents in order."""
        counts = np.zeros(self._map_shape[0], dtype=np.uint32)
        n = ctypes.c_uint64()
        self._check(self.L.fmt_map_fetch_sparse(self.h, _ptr(counts), None, 0, ctypes.byref(n)))
        entries = np.zeros(max(n.value, 1), dtype=MAP_ENTRY_DTYPE)
        self._check(self.L.fmt_map_fetch_sparse(self.h, _ptr(counts), _ptr(entries), n.value, ctypes.byref(n)))
        return counts, entries[: n.value]

    def map_pending(self, batch):
        """fmt_map_pending_run + fetch over the last sparse run: the local client's optimistic view of
        every document of `batch` (its local_ops / local_offsets, streams.MapStreamBuilder.local_*).
        Returns (counts[n_docs], status[n_docs], entries[sum(counts)]) with MAP_ENTRY_DTYPE."""
        ev = np.ascontiguousarray(batch.local_ops)
        eo = np.ascontiguousarray(batch.local_offsets, dtype=np.uint64)
        self._check(self.L.fmt_map_pending_run(self.h, _ptr(ev), len(ev), _ptr(eo)))
        counts = np.zeros(self._map_shape[0], dtype=np.uint32)
        status = np.zeros(self._map_shape[0], dtype=np.int32)
        n = ctypes.c_uint64()
        self._check(self.L.fmt_map_pending_fetch(self.h, _ptr(counts), _ptr(status), None, 0, ctypes.byref(n)))
        entries = np.zeros(max(n.value, 1), dtype=MAP_ENTRY_DTYPE)
        self._check(self.L.fmt_map_pending_fetch(self.h, _ptr(counts), _ptr(status), _ptr(entries), n.value,
                                                 ctypes.byref(n)))
        return counts, status, entries[: n.value]

    # ---- bulk legacy summaries of the last merge-tree run
    def mt_summarize_legacy(self, keys, values, chunk: int = 10000, threads: int = 0) -> dict:
        """fmt_mt_summarize_legacy: every document's legacy summary blobs (device merge + host JSON);
        returns the timing. Blobs: mt_summary(doc)."""
        from .streams import js_quote

        kq = [js_quote(k).encode("utf-8") for k in keys]
        vq = [v.encode("utf-8") for v in values]
        ka = (ctypes.c_char_p * max(len(kq), 1))(*kq)
        va = (ctypes.c_char_p * max(len(vq), 1))(*vq)
        t = FmtSummaryTiming()
        self._check(self.L.fmt_mt_summarize_legacy(self.h, ka, len(kq), va, len(vq), chunk, threads, ctypes.byref(t)))
        return {"kernel_ms": t.kernel_ms, "fetch_ms": t.fetch_ms, "format_ms": t.format_ms, "bytes": int(t.bytes),
                "threads": int(t.threads)}

    def mt_summary(self, doc: int):
        """(header, body or None) of document `doc` from the last mt_summarize_legacy."""
        h, b = ctypes.c_char_p(), ctypes.c_char_p()
        hl, bl = ctypes.c_size_t(), ctypes.c_size_t()
        self._check(self.L.fmt_mt_summary_blobs(self.h, doc, ctypes.byref(h), ctypes.byref(hl), ctypes.byref(b), ctypes.byref(bl)))
        head = ctypes.string_at(h, hl.value).decode("utf-8")
        body = ctypes.string_at(b, bl.value).decode("utf-8") if bl.value else None
        return head, body

    # ---- merge-tree
    def mt_load(self, batch):
        b, keep = batch_struct(batch)
        self._check(self.L.fmt_mt_load(self.h, ctypes.byref(b)))
        self._mt_docs = batch.n_docs

    def mt_run(self):
        self._check(self.L.fmt_mt_run(self.h))

    def mt_headers(self, raise_on_failed_docs: bool = True) -> np.ndarray:
        """Every document's result header; by default raises EngineError when a document failed
        (fmt_mt_fetch_headers returns the first failure), else returns them all."""
        out = np.zeros(self._mt_docs, dtype=DOC_RESULT_DTYPE)
        rc = self.L.fmt_mt_fetch_headers(self.h, _ptr(out))
        if raise_on_failed_docs or rc not in (FMT_OK, FMT_E_USAGE, FMT_E_DATA, FMT_E_CAPACITY, FMT_E_UNSUPPORTED):
            self._check(rc)
        return out

    def mt_doc(self, doc: int, hdr=None):
        if hdr is None:
            hdr = self.mt_headers()[doc]
        nl, nc, npp = int(hdr["n_leaves"]), int(hdr["n_chars"]), int(hdr["n_props"])
        leaves = np.zeros(max(nl, 1), dtype=LEAF_DTYPE)
        chars = np.zeros(max(nc, 1), dtype="<u2")
        props = np.zeros(max(npp, 1), dtype=PROPSET_DTYPE)
        self._check(self.L.fmt_mt_fetch_doc(self.h, doc, _ptr(leaves), nl, _ptr(chars), nc, _ptr(props), npp))
        return leaves[:nl], chars[:nc], props[:npp]

    def mt_digests(self) -> np.ndarray:
        """fmt_mt_state_digest: every document's 64-bit content digest."""
        out = np.zeros(self._mt_docs, dtype=np.uint64)
        self._check(self.L.fmt_mt_state_digest(self.h, _ptr(out)))
        return out

    def huge_profile(self, doc: int):
        """Diagnostics: shader-clock totals per phase of a huge document's last replay
        (inclusive; nested phases overlap)."""
        out = np.zeros(25, dtype=np.uint64)
        f = self.L.fmt_internal_huge_profile
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        self._check(f(self.h, doc, _ptr(out)))
        names = ["replay", "window_groups", "window_slots", "zamboni", "graduate", "load", "output", "find",
                 "scour", "pack_leaf_parent", "slot_shift", "heap", "insert", "range", "split", "pack_interior",
                 "n_group_passes", "n_slot_passes", "sum_window_entries", "sum_groups", "window_share_w0", "group_scan",
                 "text_compactions", "merge_units_in_use", "resumed_at"]
        return dict(zip(names, (int(x) for x in out)))

    def mt_remove_order(self, doc: int, hdr=None) -> np.ndarray:
        """The document's remove-order entries (fmt_mt_remove_order) of its FMT_MT_F_RMORDER ops."""
        if hdr is None:
            hdr = self.mt_headers()[doc]
        n = int(hdr["n_rm_order"])
        out = np.zeros(max(n, 1), dtype=RM_ORDER_DTYPE)
        self._check(self.L.fmt_mt_fetch_remove_order(self.h, doc, _ptr(out), n))
        return out[:n]

    def mt_legacy_props(self, doc: int, hdr=None) -> np.ndarray:
        """Per leaf, the prop-set id of getAtSeq(properties, minSeq) (what the legacy summary reads)."""
        if hdr is None:
            hdr = self.mt_headers(raise_on_failed_docs=False)[doc]
        n = int(hdr["n_leaves"])
        out = np.zeros(max(n, 1), dtype=np.uint16)
        self._check(self.L.fmt_mt_fetch_legacy_props(self.h, doc, _ptr(out), n))
        return out[:n]

    def mt_rm_clients_hi(self, doc: int, hdr=None) -> np.ndarray:
        """Per leaf, its remove clients with short ids 64..127 (bit c - 64; zero for most documents)."""
        if hdr is None:
            hdr = self.mt_headers(raise_on_failed_docs=False)[doc]
        n = int(hdr["n_leaves"])
        out = np.zeros(max(n, 1), dtype=np.uint64)
        self._check(self.L.fmt_mt_fetch_rm_clients_hi(self.h, doc, _ptr(out), n))
        return out[:n]

    def mt_rm_clients_hi2(self, doc: int, hdr=None) -> np.ndarray:
        """Per leaf, its remove clients with short ids 128..191 and 192..253 ((n, 2): bit c - 128, c - 192)."""
        if hdr is None:
            hdr = self.mt_headers(raise_on_failed_docs=False)[doc]
        n = int(hdr["n_leaves"])
        out = np.zeros(max(2 * n, 2), dtype=np.uint64)
        self._check(self.L.fmt_mt_fetch_rm_clients_hi2(self.h, doc, _ptr(out), 2 * n))
        return out[: 2 * n].reshape(n, 2)

    def mt_numbers(self, doc: int) -> np.ndarray:
        """The document's computed annotate-adjust numbers (value ids FMT_MT_VALUE_COMPUTED + index)."""
        n = ctypes.c_uint32(0)
        self._check(self.L.fmt_mt_fetch_numbers(self.h, doc, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.float64)
        if n.value:
            self._check(self.L.fmt_mt_fetch_numbers(self.h, doc, _ptr(out), n.value, ctypes.byref(n)))
        return out[: n.value]

    def mt_regen(self, doc: int):
        """f4: the document's regenerated ops (MT_OP_DTYPE) and their text after the last run
        (fmt_mt_fetch_regen; regeneratePendingOp at each reconnect record, client.ts:1452-1542)."""
        from .streams import MT_OP_DTYPE

        n, nt = ctypes.c_uint32(0), ctypes.c_uint32(0)
        self._check(self.L.fmt_mt_fetch_regen(self.h, doc, None, 0, None, 0, ctypes.byref(n), ctypes.byref(nt)))
        ops = np.zeros(max(n.value, 1), dtype=MT_OP_DTYPE)
        text = np.zeros(max(nt.value, 1), dtype="<u2")
        if n.value or nt.value:
            self._check(self.L.fmt_mt_fetch_regen(self.h, doc, _ptr(ops), n.value, _ptr(text), nt.value, ctypes.byref(n),
                                                  ctypes.byref(nt)))
        return ops[: n.value], text[: nt.value]

    def mt_catchup(self, doc: int, hdr=None) -> np.ndarray:
        """The document's catch-up ranges (fmt_mt_catchup_range) of its FMT_MT_F_CATCHUP ops."""
        if hdr is None:
            hdr = self.mt_headers()[doc]
        n = int(hdr["n_catchup"])
        out = np.zeros(max(n, 1), dtype=CATCHUP_DTYPE)
        self._check(self.L.fmt_mt_fetch_catchup(self.h, doc, _ptr(out), n))
        return out[:n]

    def mt_catchup_all(self):
        """Every document's catch-up ranges in one copy (fmt_mt_fetch_catchup_all): (offsets[n_docs + 1],
        ranges), document d's at ranges[offsets[d]:offsets[d + 1]]."""
        offs = np.zeros(self._mt_docs + 1, dtype=np.uint64)
        self._check(self.L.fmt_mt_fetch_catchup_all(self.h, _ptr(offs), None, 0))
        out = np.zeros(max(int(offs[-1]), 1), dtype=CATCHUP_DTYPE)
        self._check(self.L.fmt_mt_fetch_catchup_all(self.h, _ptr(offs), _ptr(out), int(offs[-1])))
        return offs, out[: int(offs[-1])]
