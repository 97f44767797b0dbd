"""Document sharding across GPUs: one rank per GPU, contiguous doc ranges.

Documents are independent (no cross-document op), so a multi-GPU replay is N independent replays
of contiguous document ranges balanced by op count, with nothing exchanged on the data path. The
one exchange step is at the end: every rank contributes a fixed 64-byte stats record
(`STATS_DTYPE`) to an all-gather. Over RCCL with `nccl`, or over `gloo` in the CPU tests.

`state_checksum` folds per-document result headers into one order-independent 64-bit value, so the
sum over shards equals the checksum of an unsharded replay.
"""
from __future__ import annotations

import numpy as np

from .streams import MapBatch, MergeTreeBatch

STATS_DTYPE = np.dtype(
    [
        ("rank", "<u4"),
        ("status_bad", "<u4"),   # documents whose replay failed (status != OK)
        ("doc_lo", "<u8"),
        ("doc_hi", "<u8"),
        ("ops", "<u8"),
        ("kernel_ms", "<f8"),
        ("elapsed_s", "<f8"),
        ("checksum", "<u8"),     # state_checksum of this shard's documents
        ("bytes", "<u8"),        # algorithmic bytes of this shard's launch
    ]
)
assert STATS_DTYPE.itemsize == 64


def plan_shards(doc_op_offsets: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) document ranges, one per rank, balanced by op count.

    Boundary k is the first document whose op prefix reaches k/world of all ops, so every rank
    gets within one document's ops of an equal share. Ranges cover [0, n_docs) exactly."""
    offs = np.asarray(doc_op_offsets, dtype=np.uint64)
    n_docs = len(offs) - 1
    if world < 1:
        raise ValueError("world must be >= 1")
    total = int(offs[-1])
    cuts = [0]
    for k in range(1, world):
        target = (total * k) // world
        c = int(np.searchsorted(offs, np.uint64(target), side="left"))
        cuts.append(min(max(c, cuts[-1]), n_docs))
    cuts.append(n_docs)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def slice_mt(batch: MergeTreeBatch, lo: int, hi: int) -> MergeTreeBatch:
    """Documents [lo, hi) of a merge-tree batch. Text arena and prop table are shared (ops carry
    absolute offsets into them)."""
    o0, o1 = int(batch.doc_op_offsets[lo]), int(batch.doc_op_offsets[hi])
    return MergeTreeBatch(
        ops=batch.ops[o0:o1],
        doc_op_offsets=(batch.doc_op_offsets[lo : hi + 1] - np.uint64(o0)).astype(np.uint64),
        text=batch.text,
        doc_init=batch.doc_init[lo:hi],
        props_off=batch.props_off,
        props_kv=batch.props_kv,
        keys=batch.keys,
        values=batch.values,
        clients=batch.clients[lo:hi] if batch.clients else [],
    )


def slice_map(batch: MapBatch, lo: int, hi: int) -> MapBatch:
    """Documents [lo, hi) of a SharedMap batch; doc ids are rebased to the shard."""
    o0, o1 = int(batch.doc_op_offsets[lo]), int(batch.doc_op_offsets[hi])
    ops = batch.ops[o0:o1].copy()
    ops["doc"] -= np.uint32(lo)
    return MapBatch(ops, (batch.doc_op_offsets[lo : hi + 1] - np.uint64(o0)).astype(np.uint64),
                    batch.key_bound, batch.keys, batch.values)


_HDR_FIELDS = ("status", "fail_seq", "cur_seq", "min_seq", "n_leaves", "n_chars", "n_props", "n_blocks",
               "depth", "visible_len")


def state_checksum(headers: np.ndarray, doc_lo: int = 0) -> int:
    """Order-independent checksum of per-document result headers: Σ_d mix(d, header_d) mod 2^64,
    with d the global document index, so shard checksums add up to the unsharded one."""
    n = len(headers)
    h = (np.arange(doc_lo, doc_lo + n, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        for i, f in enumerate(_HDR_FIELDS):
            v = headers[f].astype(np.int64).astype(np.uint64)
            h ^= v + np.uint64(0x632BE59BD9B4E019) * np.uint64(i + 1)
            h *= np.uint64(0xBF58476D1CE4E5B9)
            h ^= h >> np.uint64(31)
        return int(h.sum(dtype=np.uint64))


def map_checksum(slots: np.ndarray, doc_lo: int = 0) -> int:
    """Order-independent checksum of SharedMap result slots (n_docs × key_bound)."""
    nd, kb = slots.shape
    idx = (np.arange(doc_lo * kb, (doc_lo + nd) * kb, dtype=np.uint64) + np.uint64(1)).reshape(nd, kb)
    with np.errstate(over="ignore"):
        h = idx * np.uint64(0x9E3779B97F4A7C15)
        h ^= slots["value"].astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)
        h ^= slots["birth_seq"].astype(np.uint64) + np.uint64(0x94D049BB133111EB)
        h *= np.uint64(0xD6E8FEB86659FD93)
        h ^= h >> np.uint64(32)
        return int(h.sum(dtype=np.uint64))


def map_sparse_checksum(counts: np.ndarray, entries: np.ndarray, doc_lo: int = 0) -> int:
    """Order-independent checksum of sparse SharedMap entries (fmt_map_entry per live key)."""
    doc = np.repeat(np.arange(doc_lo, doc_lo + len(counts), dtype=np.uint64), counts.astype(np.int64))
    with np.errstate(over="ignore"):
        h = (doc * np.uint64(0x100000000) + entries["key"].astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        h ^= entries["value"].astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)
        h ^= entries["birth_seq"].astype(np.uint64) + np.uint64(0x94D049BB133111EB)
        h *= np.uint64(0xD6E8FEB86659FD93)
        h ^= h >> np.uint64(32)
        return int(h.sum(dtype=np.uint64))


def gather_stats(rec: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather one STATS_DTYPE record per rank (the run's single exchange step).

    `dist` is torch.distributed (initialised); `device` is "cuda" for nccl/RCCL, None for gloo."""
    import torch

    world = dist.get_world_size()
    raw = np.frombuffer(np.ascontiguousarray(rec, dtype=STATS_DTYPE).tobytes(), dtype=np.uint8)
    t = torch.from_numpy(raw.copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    out = np.concatenate([p.cpu().numpy() for p in parts])
    return np.frombuffer(out.tobytes(), dtype=STATS_DTYPE)


def digest_checksum(digests: np.ndarray, doc_lo: int = 0) -> int:
    """Order-independent fold of per-document content digests (fmt_mt_state_digest): Σ_d mix(d,
    digest_d) mod 2^64 with d the global document index, so shard sums add up to the unsharded one."""
    d = np.arange(doc_lo, doc_lo + len(digests), dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = (d + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15) ^ np.asarray(digests, dtype=np.uint64)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(31)
        return int(h.sum(dtype=np.uint64))


def gather_u64(value: int, dist, device=None) -> list[int]:
    """All-gather one unsigned 64-bit value per rank (rank order)."""
    import torch

    v = int(value) & 0xFFFFFFFFFFFFFFFF
    t = torch.tensor([v - (1 << 64) if v >= 1 << 63 else v], dtype=torch.int64)  # (two's complement bits)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.cpu().item()) & 0xFFFFFFFFFFFFFFFF for p in parts]


def combine_checksums(stats: np.ndarray) -> int:
    """Whole-job state checksum = Σ shard checksums mod 2^64."""
    return int(stats["checksum"].astype(np.uint64).sum(dtype=np.uint64))


def gather_blobs(blobs: list, dist, device=None):
    """Gatherv of variable-length byte blobs to rank 0 (the summaries the shards'
    summarizeCore would produce, shared-object-base/src/sharedObject.ts:889, end up with one
    summarizer). Every rank passes its blobs in document order; rank 0 gets all ranks' blobs in rank
    order (so in global document order for contiguous shards), the others None.

    Step 1: all-gather of each rank's (blob count, payload bytes). Step 2: every rank > 0 sends its
    blob lengths and its concatenated payload to rank 0 as one group of point-to-point ops
    (batch_isend_irecv on RCCL; isend/irecv on gloo). `device` is "cuda" for nccl, None for gloo."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    lens = np.array([len(b) for b in blobs], dtype=np.int64)
    payload = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    dev = device or "cpu"
    sizes = torch.tensor([len(blobs), payload.size], dtype=torch.int64, device=dev)
    parts = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(parts, sizes)
    sizes = [tuple(int(x) for x in p.cpu().tolist()) for p in parts]

    def p2p(ops):
        if not ops:
            return
        if device is not None:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        else:
            works = [(dist.isend if op.op is dist.isend else dist.irecv)(op.tensor, op.peer) for op in ops]
            for w in works:
                w.wait()

    if rank != 0:
        ops = []
        if len(blobs):
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(lens).to(dev), 0))
        if payload.size:
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(payload.copy()).to(dev), 0))
        p2p(ops)
        return None
    recv = {}
    ops = []
    for r in range(1, world):
        n, nb = sizes[r]
        lt = torch.empty(n, dtype=torch.int64, device=dev) if n else None
        pt = torch.empty(nb, dtype=torch.uint8, device=dev) if nb else None
        recv[r] = (lt, pt)
        if lt is not None:
            ops.append(dist.P2POp(dist.irecv, lt, r))
        if pt is not None:
            ops.append(dist.P2POp(dist.irecv, pt, r))
    p2p(ops)
    out = list(blobs)
    for r in range(1, world):
        lt, pt = recv[r]
        if lt is None:
            continue
        ln = lt.cpu().numpy()
        raw = pt.cpu().numpy().tobytes() if pt is not None else b""
        o = 0
        for k in ln:
            out.append(raw[o : o + int(k)])
            o += int(k)
    return out
