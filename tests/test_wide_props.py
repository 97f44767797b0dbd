"""Prop sets wider than one record (fmt.h FMT_MT_PROPS_KEYS_MAX = 64 keys; a set with more than
FMT_MT_PROPS_MAX = 8 takes consecutive records): segments annotated with 20-key formatting runs,
under emulation in the large tier and the huge tier == oracle (properties.ts:68-82, 135-137 have no
key limit)."""
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


def test_emulated_large_tier_wide_props(orc):
    batch = marker_batch(8, 300, seed=12, wide=20)
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        assert int(hdr[d]["status"]) == 0, d
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d])) == [], d


def test_emulated_huge_tier_wide_props(orc):
    """A T3-shaped document whose annotates carry 20-key sets and whose summary specs carry 12 keys."""
    base = workloads.t3_stream(3000, 5000, n_clients=16, max_lag=300, max_range=8, seed=13)
    n = len(base.props_off) - 1
    kv, off = [], [0]
    for c in range(n):  # props op c: 20 keys k0..k19, values by c
        kv += [(k << 16) | (1 + (c + k) % 4) for k in range(20)]
        off.append(len(kv))
    batch = dataclasses.replace(base, props_off=np.asarray(off, np.uint32), props_kv=np.asarray(kv, np.uint32),
                                keys=[f"k{k}" for k in range(20)], values=["null", "0", "1", "2", "3"])
    batch = workloads.as_legacy_load(batch, props_every=5)
    orc.set_index(True)
    try:
        segs = int(batch.snapshots[0]["n_header"]) + int(batch.snapshots[0]["n_body"])
        rc, h, lv, ch, pr, *_ = orc.mt_replay_timed(batch, 0, 0, cap_leaves=segs + 3 * len(batch.ops) + 8,
                                                    cap_chars=len(batch.text) + 8, cap_props=8192)
    finally:
        orc.set_index(False)
    assert rc == 0
    exp = (h, lv[: int(h["n_leaves"])], ch[: int(h["n_chars"])], pr[: int(h["n_props"])])
    for tiny in (False, True):
        got = emu_huge_replay(batch, tiny_groups=tiny)
        assert int(got[0]["status"]) == 0, int(got[0]["status"])
        assert compare_doc(exp, got) == []
