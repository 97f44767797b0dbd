"""Document sharding for N>1, on the CPU: shard planning, batch slicing, and a
world_size-2 gloo run whose per-shard results and gathered stats reproduce the unsharded replay.

The per-shard replay here is the oracle (test infrastructure), standing in for each rank's GPU
engine; the sharding, slicing and the single stats all-gather are the product code under test."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from fluidframework_amd import shard, workloads

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_shards_cover_and_balance():
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 4, 8):
        for n_docs in (1, 2, 7, 100, 1000):
            counts = rng.integers(0, 50, n_docs)
            offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
            plan = shard.plan_shards(offs, world)
            assert len(plan) == world
            assert plan[0][0] == 0 and plan[-1][1] == n_docs
            for (a, b), (c, _) in zip(plan, plan[1:]):
                assert a <= b == c
            total = int(offs[-1])
            for lo, hi in plan:
                ops = int(offs[hi] - offs[lo])
                assert ops <= total // world + int(counts.max(initial=0)) + 1


def test_slices_replay_like_the_whole(orc):
    batch = workloads.conflict_farm(12, n_clients=4, ops_per_doc=300, seed=9)
    rc, whole, *_ = orc.mt_replay_batch(batch, outputs=False)
    assert rc == 0
    parts = []
    for lo, hi in shard.plan_shards(batch.doc_op_offsets, 3):
        s = shard.slice_mt(batch, lo, hi)
        rc, h, *_ = orc.mt_replay_batch(s, outputs=False)
        assert rc == 0
        assert shard.state_checksum(h, lo) == shard.state_checksum(whole[lo:hi], lo)
        parts.append(shard.state_checksum(h, lo))
    assert sum(parts) % (1 << 64) == shard.state_checksum(whole)
    m = workloads.map_stream(50, 200, key_pool=20, seed=4)
    slots, _ = orc.map_replay(m)
    acc = 0
    for lo, hi in shard.plan_shards(m.doc_op_offsets, 4):
        s, _ = orc.map_replay(shard.slice_map(m, lo, hi))
        np.testing.assert_array_equal(s, slots[lo:hi])
        acc += shard.map_checksum(s, lo)
    assert acc % (1 << 64) == shard.map_checksum(slots)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist

    import oracle
    from fluidframework_amd import shard as sh, workloads as wl

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    batch = wl.conflict_farm(10, n_clients=4, ops_per_doc=200, seed=21)
    lo, hi = sh.plan_shards(batch.doc_op_offsets, world)[rank]
    rc, h, *_ = oracle.mt_replay_batch(sh.slice_mt(batch, lo, hi), outputs=False)
    rec = np.zeros(1, dtype=sh.STATS_DTYPE)
    rec["rank"], rec["doc_lo"], rec["doc_hi"] = rank, lo, hi
    rec["ops"] = int(batch.doc_op_offsets[hi] - batch.doc_op_offsets[lo])
    rec["status_bad"] = int((h["status"] != 0).sum()) + (rc != 0)
    rec["checksum"] = sh.state_checksum(h, lo)
    stats = sh.gather_stats(rec, dist)
    if rank == 0:
        np.save(out_path, stats)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shards_reproduce_unsharded(orc, tmp_path):
    out = str(tmp_path / "stats.npy")
    mp.start_processes(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    stats = np.load(out)
    assert list(stats["rank"]) == [0, 1]
    assert stats["status_bad"].sum() == 0
    batch = workloads.conflict_farm(10, n_clients=4, ops_per_doc=200, seed=21)
    assert int(stats["ops"].sum()) == len(batch.ops)
    assert stats["doc_lo"][0] == 0 and stats["doc_hi"][-1] == batch.n_docs
    assert stats["doc_hi"][0] == stats["doc_lo"][1]
    rc, whole, *_ = orc.mt_replay_batch(batch, outputs=False)
    assert shard.combine_checksums(stats) == shard.state_checksum(whole)


def test_shard_generation_equals_slicing():
    """A shard generated alone (doc_base) holds exactly the whole batch's streams for its documents."""
    whole = workloads.conflict_farm(10, n_clients=4, ops_per_doc=300, seed=7)
    part = workloads.conflict_farm(4, n_clients=4, ops_per_doc=300, seed=7, doc_base=3)
    sl = shard.slice_mt(whole, 3, 7)
    keys = ("seq", "ref_seq", "min_seq", "pos1", "pos2", "len", "client", "type")
    for k in keys:
        assert np.array_equal(part.ops[k], sl.ops[k]), k
    ins = part.ops["type"] == 0
    for i in np.nonzero(ins)[0][:200]:
        a, b = int(part.ops["payload"][i]), int(sl.ops["payload"][i])
        n = int(part.ops["len"][i])
        assert np.array_equal(part.text[a : a + n], whole.text[b : b + n])


def _gather_main(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    import torch.distributed as dist

    from fluidframework_amd import shard as sh

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    # rank 1 has no blobs; rank 2 has an empty blob among others
    mine = {0: [b"a", b"bc" * 1000], 1: [], 2: [b"", "é€😀".encode(), b"\0x"]}[rank]
    out = sh.gather_blobs(mine, dist)
    if rank == 0:
        with open(out_path, "wb") as f:
            for b in out:
                f.write(len(b).to_bytes(8, "little") + b)
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_blobs_world3(tmp_path):
    out = str(tmp_path / "blobs.bin")
    mp.start_processes(_gather_main, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    raw = open(out, "rb").read()
    got, o = [], 0
    while o < len(raw):
        n = int.from_bytes(raw[o : o + 8], "little")
        got.append(raw[o + 8 : o + 8 + n])
        o += 8 + n
    assert got == [b"a", b"bc" * 1000, b"", "é€😀".encode(), b"\0x"]


def _u64_main(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    import torch.distributed as dist

    from fluidframework_amd import shard as sh

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    vals = [0xFFFFFFFFFFFFFFFF, 0x8000000000000000, 12345]
    got = sh.gather_u64(vals[rank], dist)
    if rank == 0:
        np.save(out_path, np.array(got, dtype=np.uint64))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_u64_world3_and_digest_fold(tmp_path):
    """The whole-job content digest: per-rank folds of the per-document digests, all-gathered as
    unsigned 64-bit values, add up to the unsharded fold."""
    out = str(tmp_path / "u64.npy")
    mp.start_processes(_u64_main, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    assert [int(x) for x in np.load(out)] == [0xFFFFFFFFFFFFFFFF, 0x8000000000000000, 12345]
    dig = np.random.default_rng(3).integers(0, 2**63, 50, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    parts = [shard.digest_checksum(dig[lo:hi], lo) for lo, hi in shard.plan_shards(np.arange(51, dtype=np.uint64), 4)]
    assert sum(parts) & 0xFFFFFFFFFFFFFFFF == shard.digest_checksum(dig)
