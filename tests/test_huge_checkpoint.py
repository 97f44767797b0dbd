"""Large → huge as a checkpoint, not a restart (huge_ckpt.h).

A plain document the large tier is about to outgrow (2048 leaves, 131,071 UTF-16 units, its last
blocks or prop sets, a writer past 63) stops before that op: the large tier writes its result slabs
and a record of what they do not carry — the exact B+tree with its block ids, leaf ids, the LRU heap
in array order, the free-block list, the collab window, catch-up count and live obliterates — and the
huge tier rebuilds that tree in its paged layout and replays on from that op (`HugeDoc::loadFromLarge`).
The reference grows one tree without bound (insertSegments, mergeTree.ts:1484-1517), so the result
must equal the oracle's whole replay bit for bit: every leaf field (block ordinals and depth
included, which only an exact tree reproduces), the text, the prop sets, the catch-up ranges.

CPU: the large tier and the huge tier under host emulation (`emu_grow_replay`); GPU: the runtime
path, with `huge_profile()["resumed_at"]` showing the op the huge tier resumed at (not 0).
"""
import numpy as np
import pytest

from fluidframework_amd import native
from fluidframework_amd.streams import MT_F_CATCHUP, MT_INSERT, MT_OBLITERATE, MergeTreeStreamBuilder
from growth import growth_batch, growth_messages
from mt_compare import compare_doc, emu_grow_replay

CAP_CU = 1 << 15


def _oracle(orc, batch, cap_catchup=0):
    r = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=4096, cap_catchup=cap_catchup)
    assert r[0] == 0
    return r


def _exp(r, d):
    oh, ol, oc, op = r[1], r[2], r[3], r[4]
    h = oh[d]
    return h, ol[d][: int(h["n_leaves"])], oc[d][: int(h["n_chars"])], op[d][: int(h["n_props"])]


def _ob_growth(seed=21, n_ops=900):
    """A document near the large tier's text limit that crosses it while obliterates are live."""
    import random

    rnd = random.Random(seed)
    init = "".join(rnd.choice("abcdefgh") for _ in range(128000))
    b = MergeTreeStreamBuilder()
    d = b.begin_doc(init, observer="observer")
    length = len(init)
    for seq in range(1, n_ops + 1):
        c = f"w{rnd.randrange(5)}"
        if rnd.random() < 0.2 and length > 200:
            a = rnd.randrange(length - 10)
            op = {"type": MT_OBLITERATE, "pos1": a, "pos2": a + rnd.randint(1, 6)}
            length -= op["pos2"] - op["pos1"]
        else:
            s = "".join(rnd.choice("XYZ") for _ in range(rnd.randint(3, 12)))
            op = {"type": MT_INSERT, "pos1": rnd.randrange(length + 1), "seg": s}
            length += len(s)
        d.add_message({"clientId": c, "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                       "minimumSequenceNumber": max(0, seq - 40), "type": "op", "contents": op})
    return b.finish()


@pytest.fixture(scope="module")
def grown():
    return growth_batch([("", 4700, 11), ("xyz" * 100, 4700, 12)])


def test_emulated_large_tier_checkpoints_and_huge_tier_resumes(orc, grown):
    r = _oracle(orc, grown)
    got, resumed = emu_grow_replay(grown)
    for d in range(grown.n_docs):
        assert resumed[d] > 0, d  # (the large tier stopped there; ops before it were not replayed again)
        assert int(got[d][0]["status"]) == 0
        assert compare_doc(_exp(r, d), got[d]) == [], d
    assert (r[1]["n_chars"] > 131071).all()


def test_emulated_checkpoint_with_tiny_groups(orc, grown):
    """The resumed tree in 16-slot groups (a group split on the first inserts after the resume)."""
    r = _oracle(orc, grown)
    got, resumed = emu_grow_replay(grown, tiny_groups=True)
    for d in range(grown.n_docs):
        assert resumed[d] > 0
        assert compare_doc(_exp(r, d), got[d]) == [], d


def test_emulated_checkpoint_carries_catchup_ranges(orc):
    """Every op flagged for catch-up: the ranges the large tier recorded before the checkpoint stay,
    the huge tier appends its own after them."""
    batch = growth_batch([("", 4700, 13)])
    batch.ops["flags"] |= MT_F_CATCHUP
    r = _oracle(orc, batch, cap_catchup=CAP_CU)
    got, resumed = emu_grow_replay(batch, cap_catchup=CAP_CU)
    assert resumed[0] > 0
    assert compare_doc(_exp(r, 0), got[0][:4]) == []
    n = int(r[1][0]["n_catchup"])
    assert int(got[0][0]["n_catchup"]) == n
    assert np.array_equal(r[6][0][:n], got[0][4][:n])


def test_emulated_checkpoint_with_live_obliterates(orc):
    batch = _ob_growth()
    r = _oracle(orc, batch)
    got, resumed = emu_grow_replay(batch)
    assert resumed[0] > 0
    assert int(got[0][0]["status"]) == 0
    assert compare_doc(_exp(r, 0), got[0]) == []


def _relpos_growth():
    """A marker-rich document with legacy relativePos1 inserts that outgrows the large tier (its prop
    sets: every Marker's markerId is its own set) — round 6: relative-position batches checkpoint too."""
    from marker_docs import marker_batch

    return marker_batch(1, 6000, seed=2)


def test_emulated_checkpoint_with_relative_positions(orc):
    batch = _relpos_growth()
    r = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1 << 15)
    assert r[0] == 0
    got, resumed = emu_grow_replay(batch)
    assert resumed[0] > 0
    assert int(got[0][0]["status"]) == 0
    assert compare_doc(_exp(r, 0), got[0]) == []


@pytest.mark.gpu
def test_relative_position_document_resumes_in_the_huge_tier_on_gpu(orc):
    batch = _relpos_growth()
    r = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1 << 15)
    assert r[0] == 0
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        assert int(hdrs[0]["status"]) == 0
        lv, ch, pr = eng.mt_doc(0, hdrs[0])
        assert compare_doc(_exp(r, 0), (hdrs[0], lv, ch, pr)) == []
        assert eng.huge_profile(0)["resumed_at"] > 0
    finally:
        eng.close()


def _rm_growth():
    """A growing document with remove-order recording (FMT_MT_F_RMORDER on every op) and overlapping
    removes — after most removes a dedicated writer removes the same range from the same refSeq —
    that crosses the large tier at op 4527 and ends 10 ops later, so removes from before the
    checkpoint are still above the final minSeq and their later stamps are entries the large tier
    recorded (without the carried count the emulated stamp lists lose them)."""
    import random

    from growth import growth_messages

    from fluidframework_amd.streams import MergeTreeStreamBuilder, flag_remove_order
    rnd = random.Random(112)
    seqmap, out, last_dup = {0: 0}, [], 0
    for m in growth_messages(n_ops=4700, seed=13):
        s = len(out) + 1
        seqmap[m["sequenceNumber"]] = s
        ref, msn = seqmap[m["referenceSequenceNumber"]], seqmap[m["minimumSequenceNumber"]]
        out.append(dict(m, sequenceNumber=s, referenceSequenceNumber=ref, minimumSequenceNumber=msn))
        # (the same view and range: the visible length does not change, so later positions stand)
        if m["contents"]["type"] == 1 and ref >= last_dup and rnd.random() < 0.7:
            out.append(dict(m, clientId="wd", sequenceNumber=s + 1, referenceSequenceNumber=ref, minimumSequenceNumber=msn))
            last_dup = s + 1
    b = MergeTreeStreamBuilder()
    d = b.begin_doc("", observer="observer")
    for m in out[:4537]:
        d.add_message(m)
    batch = b.finish()
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    return batch


def test_emulated_checkpoint_with_remove_order(orc):
    from test_huge_emulated import _oracle_doc, _removers_match

    batch = _rm_growth()
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got, resumed = emu_grow_replay(batch, cap_rm=1 << 16)
    assert resumed[0] > 0
    assert int(got[0][0]["status"]) == 0
    assert compare_doc(exp, got[0][:4]) == []
    assert _removers_match(orc, batch, got[0], got[0][4]) > 0


@pytest.mark.gpu
def test_remove_order_document_resumes_in_the_huge_tier_on_gpu(orc):
    from test_huge_emulated import _oracle_doc, _removers_match

    batch = _rm_growth()
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        assert int(hdrs[0]["status"]) == 0
        lv, ch, pr = eng.mt_doc(0, hdrs[0])
        assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
        assert eng.huge_profile(0)["resumed_at"] > 0
        rm = eng.mt_remove_order(0, hdrs[0])
        assert _removers_match(orc, batch, (hdrs[0], lv), rm) > 0
    finally:
        eng.close()


def _adjust_growth():
    """A marker-rich document whose annotates adjust "weight", past the large tier — round 6:
    annotate-adjust batches checkpoint too (the PropertiesManager records and computed numbers stay in
    their slabs; the record carries the record count). The stream ends two ops after the checkpoint
    (op 2097), so adjusts from before it are still above the final minSeq and the legacy getAtSeq view
    reads their records (without the carried count it differs from the oracle's)."""
    from marker_docs import marker_batch

    return marker_batch(1, 2099, seed=5, adjust=True)


def _adjust_oracle(orc, batch):
    nums = []
    orc.set_index(True)
    try:
        r = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1 << 15, numbers=nums)
    finally:
        orc.set_index(False)
    assert r[0] == 0
    return r, nums[0], orc.mt_replay_summary(batch, 0, batch.keys, batch.values)


def test_emulated_checkpoint_with_annotate_adjust(orc):
    from fluidframework_amd.summary import legacy_summary, values_with_numbers

    batch = _adjust_growth()
    r, want_nums, want = _adjust_oracle(orc, batch)
    got, resumed = emu_grow_replay(batch)
    assert resumed[0] > 0
    h, lv, ch, pr, legacy, nums = got[0]
    assert int(h["status"]) == 0
    assert compare_doc(_exp(r, 0), (h, lv, ch, pr)) == []
    assert np.array_equal(nums, want_nums)
    vals = values_with_numbers(batch.values, nums)
    assert legacy_summary(h, lv, ch, pr, batch.keys, vals, legacy_props=legacy) == want


@pytest.mark.gpu
def test_annotate_adjust_document_resumes_in_the_huge_tier_on_gpu(orc):
    from fluidframework_amd.summary import legacy_summary, values_with_numbers

    batch = _adjust_growth()
    r, want_nums, want = _adjust_oracle(orc, batch)
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        assert int(hdrs[0]["status"]) == 0
        lv, ch, pr = eng.mt_doc(0, hdrs[0])
        assert compare_doc(_exp(r, 0), (hdrs[0], lv, ch, pr)) == []
        assert eng.huge_profile(0)["resumed_at"] > 0
        got_nums = eng.mt_numbers(0)
        assert np.array_equal(got_nums, want_nums)
        eng.mt_summarize_legacy(batch.keys, batch.values)
        assert eng.mt_summary(0) == want
        vals = values_with_numbers(batch.values, got_nums)
        assert legacy_summary(hdrs[0], lv, ch, pr, batch.keys, vals,
                              legacy_props=eng.mt_legacy_props(0, hdrs[0])) == want
    finally:
        eng.close()


@pytest.mark.gpu
def test_large_to_huge_checkpoint_on_gpu(orc, grown):
    """Through the runtime: the grown documents resume in the huge tier at the large tier's stop and
    equal the oracle; the ordinary documents beside them replay as before."""
    from growth import growth_batch as gb
    from fluidframework_amd import workloads
    from test_gpu_huge import _concat

    farm = workloads.conflict_farm(16, n_clients=8, ops_per_doc=600, seed=3)
    batch = _concat([farm, grown, _ob_growth(), farm])
    r = _oracle(orc, batch)
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        for d in range(batch.n_docs):
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            assert compare_doc(_exp(r, d), (hdrs[d], lv, ch, pr)) == [], d
        for d in range(farm.n_docs, farm.n_docs + 3):
            assert eng.huge_profile(d)["resumed_at"] > 0, d
    finally:
        eng.close()
