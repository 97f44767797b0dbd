"""Prop sets wider than one record (fmt.h FMT_MT_PROPS_KEYS_MAX = 128 keys, 64 until round 6; a set
with more than FMT_MT_PROPS_MAX = 8 takes consecutive records): segments annotated with 20-key and
128-key formatting runs, under emulation in the large tier and the huge tier == oracle
(properties.ts:68-82, 135-137 have no key limit)."""
import pytest
import dataclasses

import numpy as np

from fluidframework_amd import workloads
from fluidframework_amd.native import PROPS_CONT, propset_entries
from marker_docs import marker_batch
from mt_compare import compare_doc, emu_caps, emu_huge_replay, emu_replay


def test_wide_sets_take_consecutive_records(orc):
    batch = marker_batch(6, 300, seed=11, wide=20)
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    widths = [len(propset_entries(op[d], int(p))) for d in range(6) for p in ol[d]["props"][: int(oh[d]["n_leaves"])]
              if int(p) != 0xFFFF]
    assert max(widths) > 16
    assert (op[0]["n"][: int(oh[0]["n_props"])] == PROPS_CONT).any()


@pytest.mark.parametrize("wide,n_ops", [(20, 300), (122, 200)])
def test_emulated_large_tier_wide_props(orc, wide, n_ops):
    """20-key runs, and runs of 122 of 128 keys (their unions stay within FMT_MT_PROPS_KEYS_MAX; sets
    of up to 16 records, null deletes shifting entries across the working set's 64-slot chunks)."""
    batch = marker_batch(8, n_ops, seed=12, wide=wide)
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        assert int(hdr[d]["status"]) == 0, d
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d])) == [], d
    widths = [len(propset_entries(op[d], int(p))) for d in range(batch.n_docs)
              for p in ol[d]["props"][: int(oh[d]["n_leaves"])] if int(p) != 0xFFFF]
    assert max(widths) > (64 if wide > 64 else 16)


def _t3_wide(wide):
    """A T3-shaped document whose annotates carry `wide`-key sets and whose summary specs carry 12 keys;
    past 64 keys every third annotate nulls the keys of one residue class, so sets shrink and grow
    across the working set's 64-slot chunk boundary."""
    base = workloads.t3_stream(3000, 5000, n_clients=16, max_lag=300, max_range=8, seed=13)
    n = len(base.props_off) - 1
    kv, off = [], [0]
    for c in range(n):  # props op c: `wide` keys, values by c (past 64 wide: some of them nulls)
        kv += [(k << 16) | (0 if wide > 64 and c % 3 == 2 and k % 5 == c % 5 else 1 + (c + k) % 4) for k in range(wide)]
        off.append(len(kv))
    batch = dataclasses.replace(base, props_off=np.asarray(off, np.uint32), props_kv=np.asarray(kv, np.uint32),
                                keys=[f"k{k}" for k in range(wide)], values=["null", "0", "1", "2", "3"])
    return workloads.as_legacy_load(batch, props_every=5)


def _t3_oracle(orc, batch):
    orc.set_index(True)
    try:
        segs = int(batch.snapshots[0]["n_header"]) + int(batch.snapshots[0]["n_body"])
        rc, h, lv, ch, pr, *_ = orc.mt_replay_timed(batch, 0, 0, cap_leaves=segs + 3 * len(batch.ops) + 8,
                                                    cap_chars=len(batch.text) + 8, cap_props=1 << 16)
    finally:
        orc.set_index(False)
    assert rc == 0
    return h, lv[: int(h["n_leaves"])], ch[: int(h["n_chars"])], pr[: int(h["n_props"])]


@pytest.mark.parametrize("wide", [20, 128])
def test_emulated_huge_tier_wide_props(orc, wide):
    batch = _t3_wide(wide)
    exp = _t3_oracle(orc, batch)
    if wide > 64:
        assert max(len(propset_entries(exp[3], int(p))) for p in exp[1]["props"] if int(p) != 0xFFFF) > 64
    for tiny in (False, True):
        got = emu_huge_replay(batch, tiny_groups=tiny)
        assert int(got[0]["status"]) == 0, int(got[0]["status"])
        assert compare_doc(exp, got) == []


@pytest.mark.gpu
def test_128_key_sets_on_gpu(orc):
    """On the GPU: the 128-key T3-shaped document (huge tier) and conflict documents with runs of 122
    of 128 keys (the compact → small → large cascade) == oracle, with state digests."""
    from fluidframework_amd import native

    e = native.Engine(0)
    try:
        batch = _t3_wide(128)
        exp = _t3_oracle(orc, batch)
        e.mt_load(batch)
        e.mt_run()
        h = e.mt_headers()[0]
        assert int(h["status"]) == 0
        assert compare_doc(exp, (h,) + tuple(e.mt_doc(0, h))) == []
        batch = marker_batch(64, 200, seed=22, wide=122)
        e.mt_load(batch)
        e.mt_run()
        hdrs = e.mt_headers()
        assert (hdrs["status"] == 0).all()
        cl, cc, cp = emu_caps(True)
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
        assert rc == 0
        for d in range(batch.n_docs):
            assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d],) + tuple(e.mt_doc(d, hdrs[d]))) == [], d
        rc, odig, _, _ = orc.mt_replay_digest(batch, threads=8)
        assert rc == 0
        assert np.array_equal(e.mt_digests(), odig)
    finally:
        e.close()
