"""A T3-shaped document loaded from a SnapshotV1-style summary whose header segments carry merge info
above minSeq (tests only): the stream's seqs move up by K so that the summary is taken at seq K with
minSeq K - 40; every 40th segment is inserted above minSeq by a writer, and a removed segment
(remove stamps of one to three writers above minSeq, setRemove and sliceRemove) follows every 25th.
Every op's refSeq is >= K, so the inserted segments are visible and the removed ones invisible in
every perspective the ops use: the generated positions stay valid."""
import dataclasses

import numpy as np

from fluidframework_amd.streams import NON_COLLAB_CLIENT, SNAPSHOT_INFO_DTYPE, SNAPSHOT_SEG_DTYPE, STAMP_DTYPE


def with_v1_merge_info(batch, k: int = 100, seed: int = 1):
    rng = np.random.default_rng(seed)
    ops = batch.ops.copy()
    ops["seq"] += k
    ops["ref_seq"] += k
    ops["min_seq"] += k
    snaps = batch.snapshots.copy()
    snaps["seq"], snaps["min_seq"] = k, k - 40
    old = batch.snapshot_segs
    segs, info, stamps = [], [], []
    for j in range(len(old)):
        s = old[j]
        if j % 40 == 7:  # inserted above minSeq by writer 1..20
            info.append((int(rng.integers(k - 39, k + 1)), int(rng.integers(1, 21)), 0, 0))
        else:
            info.append((0, NON_COLLAB_CLIENT, 0, 0))
        segs.append(tuple(s))
        if j % 25 == 3:  # a tombstone removed above minSeq
            n = int(rng.integers(1, 4))
            seqs = sorted(int(x) for x in rng.integers(k - 39, k + 1, size=n))
            first = len(stamps)
            clients = rng.choice(np.arange(1, 30), size=n, replace=False)
            for t in range(n):
                stamps.append((seqs[t], int(clients[t]), int(rng.integers(0, 2)), 0))
            ins = int(rng.integers(1, k - 40)) if rng.random() < 0.5 else 0
            info.append((ins, int(rng.integers(1, 21)) if ins else NON_COLLAB_CLIENT, first, n))
            segs.append((int(s["text"]), int(s["len"]), 0xFFFFFFFF))
    snaps["n_header"], snaps["n_body"] = len(segs), 0
    return dataclasses.replace(batch, ops=ops, snapshots=snaps, snapshot_segs=np.array(segs, dtype=SNAPSHOT_SEG_DTYPE),
                               snapshot_info=np.array(info, dtype=SNAPSHOT_INFO_DTYPE),
                               snapshot_stamps=np.array(stamps, dtype=STAMP_DTYPE))
