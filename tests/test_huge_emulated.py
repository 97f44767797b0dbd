"""The huge-document engine (csrc/huge_engine.h: paged leaf blocks, group lists, window table —
the T3 path, BASELINE config 5) under host emulation, bit-exact against the oracle on T3-shaped
documents: every leaf field, the text, the prop sets and the header."""
import numpy as np
import pytest

from fluidframework_amd import workloads
from mt_compare import compare_doc, emu_huge_replay


def _oracle_doc(orc, batch, cap_props=4096):
    orc.set_index(True)
    try:
        sd = batch.snapshots[0] if batch.snapshots is not None else None
        segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None else 1
        nops = len(batch.ops)
        rc, h, lv, ch, pr, *_ = orc.mt_replay_timed(batch, 0, 0, cap_leaves=segs + 3 * nops + 8,
                                                    cap_chars=len(batch.text) + 8, cap_props=cap_props)
    finally:
        orc.set_index(False)
    return rc, (h, lv[: int(h["n_leaves"])], ch[: int(h["n_chars"])], pr[: int(h["n_props"])])


@pytest.mark.parametrize("segs,ops,clients,lag,rng,seed,tiny", [
    (200, 300, 4, 16, 8, 1, False),
    (2000, 3000, 16, 300, 8, 2, False),
    (5000, 8000, 63, 4096, 8, 3, False),
    (30000, 20000, 63, 4096, 40, 4, False),
    (3000, 6000, 31, 500, 8, 5, True),
    (2000, 8000, 63, 2000, 200, 6, True),
    (700, 12000, 8, 64, 30, 7, True),
])
def test_huge_engine_matches_oracle(orc, segs, ops, clients, lag, rng, seed, tiny):
    batch = workloads.t3_stream(segs, ops, n_clients=clients, max_lag=lag, max_range=rng, seed=seed)
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=tiny)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, got) == []


def test_huge_engine_prop_sets_in_other_key_order_match(orc):
    """matchProperties ignores key order: clients 2k and 2k+1 annotate {a, b} with the same values in
    opposite key orders, so zamboni appends across their leaves (the engine's prop match classes;
    comparing prop set ids instead makes this case differ from the oracle)."""
    import dataclasses

    import numpy as np

    from fluidframework_amd.streams import js_json
    batch = workloads.t3_stream(300, 20000, n_clients=4, max_lag=64, max_range=100, seed=1)
    n = len(batch.props_off) - 1
    kv = []
    for c in range(n):
        pa, pb = (0 << 16) | (1 + (c // 2) % 3), (1 << 16) | 1
        kv += [pa, pb] if c % 2 == 0 else [pb, pa]
    batch = dataclasses.replace(batch, props_off=np.arange(0, 2 * n + 1, 2, dtype=np.uint32),
                                props_kv=np.array(kv, dtype=np.uint32), keys=["a", "b"],
                                values=["null"] + [js_json(i) for i in range(8)])
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    for tiny in (False, True):
        got = emu_huge_replay(batch, tiny_groups=tiny)
        assert int(got[0]["status"]) == 0
        assert compare_doc(exp, got) == []


def test_huge_engine_inserts_with_props(orc):
    """seg {text, props} inserts (TextSegment.make(text, props)) in a huge document."""
    batch = workloads.with_insert_props(workloads.t3_stream(3000, 8000, n_clients=16, max_lag=300, max_range=8, seed=9))
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=True)
    assert int(got[0]["status"]) == 0
    assert compare_doc(exp, got) == []


def test_huge_engine_loaded_markers(orc):
    """A huge document whose summary holds Marker segments (every third 1-unit spec becomes one, so
    the generated ops' positions stay valid; its arena unit is the refType): markers never append in
    zamboni and keep their flag through the replay."""
    import dataclasses

    import numpy as np

    from fluidframework_amd.streams import MT_LEAF_MARKER, MT_SEG_MARKER
    batch = workloads.t3_stream(4000, 8000, n_clients=16, max_lag=300, max_range=8, seed=5)
    segs = batch.snapshot_segs.copy()
    idx = np.nonzero(segs["len"] == 1)[0][::3]
    segs["len"][idx] = 1 | MT_SEG_MARKER
    batch = dataclasses.replace(batch, snapshot_segs=segs)
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=True)
    assert int(got[0]["status"]) == 0
    assert compare_doc(exp, got) == []
    assert int((exp[1]["pad"] & MT_LEAF_MARKER != 0).sum()) > 50


def test_huge_engine_merge_area_compaction(orc, monkeypatch, capfd):
    """A tight merge area (4x the document's text) on a T3-shaped document with 16-slot groups: the
    merge area compacts into its other half, walking every group, and the state still == oracle."""
    import re

    batch = workloads.t3_stream(3000, 6000, n_clients=31, max_lag=500, max_range=8, seed=5)
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    doc_chars = int(batch.snapshot_segs["len"].sum()) + int(batch.ops["len"][batch.ops["type"] == 0].sum())
    monkeypatch.setenv("FMT_EMU_TEXTCAP", str(len(batch.text) + 4 * doc_chars + 64))
    got = emu_huge_replay(batch, tiny_groups=True)
    assert int(re.search(r"compactions (\d+)", capfd.readouterr().err).group(1)) >= 1
    assert int(got[0]["status"]) == 0
    assert compare_doc(exp, got) == []


@pytest.mark.parametrize("segs,ops,props_every,tiny,seed", [
    (3000, 4000, 0, False, 11),
    (6000, 8000, 3, True, 12),
    (20000, 6000, 7, False, 13),
])
def test_huge_engine_legacy_header_and_body(orc, segs, ops, props_every, tiny, seed):
    """A summary in SnapshotLegacy.emit's shape — a header chunk of ~10,000 units, the rest in the
    body chunk appended by loadBody (snapshotLoader.ts:277-309) — with props on some segment specs:
    the tree the appends build (4 / 4 splits up the right edge) and every replayed op == oracle."""
    batch = workloads.as_legacy_load(workloads.t3_stream(segs, ops, n_clients=16, max_lag=300, max_range=8, seed=seed),
                                     props_every=props_every)
    assert int(batch.snapshots[0]["n_body"]) > 0
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=tiny)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, got) == []


def test_huge_engine_body_only_load_and_shape(orc):
    """The loaded tree alone (no ops) for header+body splits at several sizes, including an empty
    header (the body's first append makes the empty root the leaf block): block ordinals and depth."""
    import dataclasses

    import numpy as np
    base = workloads.t3_stream(5000, 1, n_clients=2, max_lag=1, seed=3)
    for n_header in (0, 1, 7, 8, 49, 50, 343, 344, 2222):
        snaps = base.snapshots.copy()
        snaps["n_header"], snaps["n_body"] = n_header, 5000 - n_header
        batch = dataclasses.replace(base, snapshots=snaps, ops=base.ops[:0],
                                    doc_op_offsets=np.array([0, 0], dtype=np.uint64))
        rc, exp = _oracle_doc(orc, batch)
        assert rc == 0
        got = emu_huge_replay(batch)
        assert int(got[0]["status"]) == 0
        assert compare_doc(exp, got) == [], n_header


def test_huge_engine_zamboni_empties_the_root(orc):
    """Zamboni scours every block of a document one remove emptied; packParent leaves the root
    childless (zamboni.ts:129-132) and the next insert makes it the leaf block again."""
    batch = workloads.emptying_stream(3000, 600, seed=4)
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    for tiny in (False, True):
        got = emu_huge_replay(batch, tiny_groups=tiny)
        assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
        assert compare_doc(exp, got) == []


@pytest.mark.parametrize("segs,ops,rng,tiny,seed,legacy", [
    (3000, 6000, 8, True, 31, False),
    (8000, 8000, 200, False, 32, True),
])
def test_huge_engine_catchup_ranges(orc, segs, ops, rng, tiny, seed, legacy):
    """Catch-up ranges (sequence.ts:395-452) of the ops a legacy summary keeps (seq above the final
    minSeq, refSeq != seq - 1: streams.flag_catchup), recorded by the huge engine == oracle."""
    import numpy as np

    from fluidframework_amd.streams import MT_F_CATCHUP, flag_catchup
    batch = workloads.t3_stream(segs, ops, n_clients=31, max_lag=1500, max_range=rng, seed=seed)
    if legacy:
        batch = workloads.as_legacy_load(batch, props_every=4)
    flag_catchup(batch.ops, batch.doc_op_offsets)
    n_flag = int(((batch.ops["flags"] & MT_F_CATCHUP) != 0).sum())
    assert n_flag > 100
    cap = 16 * n_flag + 16
    n_segs = int(batch.snapshots[0]["n_header"]) + int(batch.snapshots[0]["n_body"])
    orc.set_index(True)
    try:
        rc, oh, olv, och, opr, _, ocu = orc.mt_replay_batch(batch, cap_leaves=n_segs + 3 * ops + 8, cap_chars=len(batch.text) + 8,
                                                           cap_props=4096, cap_catchup=cap)
    finally:
        orc.set_index(False)
    assert rc == 0
    h = oh[0]
    exp = (h, olv[0][: int(h["n_leaves"])], och[0][: int(h["n_chars"])], opr[0][: int(h["n_props"])])
    *got, cu = emu_huge_replay(batch, tiny_groups=tiny, cap_catchup=cap)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, tuple(got)) == []
    assert int(h["n_catchup"]) > n_flag // 2
    assert np.array_equal(cu, ocu[0][: int(h["n_catchup"])])


def _removers_match(orc, batch, got, rm):
    import sys

    from fluidframework_amd import summary

    h, lv = got[0], got[1]
    want = orc.mt_removers(batch, 0)
    ops = batch.ops[int(batch.doc_op_offsets[0]) : int(batch.doc_op_offsets[1])]
    mine = summary.removers_from_engine(lv, int(h["n_leaves"]), rm, ops)
    ms, multi = int(h["min_seq"]), 0
    for i in range(int(h["n_leaves"])):
        r = int(lv[i]["rm_seq"])
        if r != summary.NOT_REMOVED and r > ms:
            assert mine.get(i) == want.get(i), (i, mine.get(i), want.get(i))
            multi += len(want[i]) > 1
    return multi


@pytest.mark.parametrize("tiny", [False, True])
def test_huge_engine_remove_order(orc, tiny):
    """Remove-order entries (SnapshotV1's removedClientIds order, snapshotV1.ts:207-265) recorded by
    the huge engine for the REMOVEs above the final minSeq: every leaf's stamp list == the oracle's."""
    from fluidframework_amd.streams import flag_remove_order
    batch = workloads.t3_stream(3000, 8000, n_clients=31, max_lag=600, max_range=60, seed=41)
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=tiny, cap_rm=1 << 16)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, got[:4]) == []
    assert int(got[0]["n_rm_order"]) > 0
    assert _removers_match(orc, batch, got, got[4]) > 0


def test_huge_engine_remove_order_with_obliterates(orc):
    """The same with obliterates (sliceRemove stamps, obliterate-on-insert) on a farm past the large
    tier (135,000-unit initial text)."""
    from test_huge_obliterate import _one
    from test_obliterate import long_obliterate_farms

    from fluidframework_amd.streams import flag_remove_order
    for doc in (0, 4):
        one = _one(long_obliterate_farms(extra=135000), doc)
        flag_remove_order(one.ops, one.doc_op_offsets)
        got = emu_huge_replay(one, 0, cap_rm=1 << 16)
        assert int(got[0]["status"]) == 0, doc
        _removers_match(orc, one, got, got[4])


@pytest.mark.parametrize("tiny", [False, True])
def test_huge_engine_v1_merge_info_load(orc, tiny):
    """A huge document loaded from a SnapshotV1 summary whose header segments carry merge info above
    minSeq (specToSegment's insert and remove stamps, snapshotLoader.ts:105-175): those leaves enter
    the window table at load, and the replay == oracle."""
    from v1_huge import with_v1_merge_info
    batch = with_v1_merge_info(workloads.t3_stream(4000, 6000, n_clients=31, max_lag=800, max_range=8, seed=51))
    rc, exp = _oracle_doc(orc, batch)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=tiny)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, got) == []


def marker_reload(orc, n_ops, split, seed):
    """A marker-rich document (marker_docs) summarized by the oracle after `split` messages (legacy
    header/body + catch-up blob) and reloaded, the rest of its messages after it: relative positions
    then name Markers loaded from the summary as well as inserted ones."""
    from marker_docs import doc_messages

    from fluidframework_amd import summary
    from fluidframework_amd.streams import MergeTreeStreamBuilder
    init, msgs = doc_messages(0, n_ops, seed)
    b = MergeTreeStreamBuilder(keep_messages=True)
    doc = b.begin_doc(init)
    for m in msgs[:split]:
        doc.add_message(m)
    first = b.finish(catchup=True)
    rc, h, lv, ch, pr, _, cu = orc.mt_replay_batch(first, cap_leaves=4 * split + 64, cap_chars=len(first.text) + 8,
                                                 cap_props=1 << 14, cap_catchup=4 * split + 64)
    assert rc == 0
    head, body = summary.legacy_summary(h[0], lv[0], ch[0], pr[0], first.keys, first.values, chunk_size=200)
    blob = summary.catchup_blob(summary.catchup_messages(first.messages[0], cu[0][: h[0]["n_catchup"]],
                                                         int(h[0]["min_seq"])))
    b2 = MergeTreeStreamBuilder()
    doc = b2.begin_doc_from_summary(head, body, blob)
    for m in msgs[split:]:
        doc.add_message(m)
    return b2.finish()


@pytest.mark.parametrize("n_ops,split,seed,tiny", [(3000, 0, 1, True), (6000, 0, 2, False), (5000, 2500, 3, True),
                                                   (8000, 6000, 4, False), (12000, 0, 5, False)])
def test_huge_engine_relative_positions(orc, n_ops, split, seed, tiny):
    """Legacy relativePos1 inserts (getValidOpRange, client.ts:758-767) in a huge document: the
    marker named by markerId found through the document's marker list (inserted Markers, and with a
    split the ones loaded from the summary), positioned in the op's view (posFromRelativePos,
    mergeTree.ts:1462-1483). The longest document interns more than 4096 prop sets (every Marker's
    markerId is its own set: the hash-table interning, past the LDS class cache)."""
    from marker_docs import marker_batch
    from fluidframework_amd.streams import MT_F_REL1
    batch = marker_batch(1, n_ops, seed=seed) if split == 0 else marker_reload(orc, n_ops, split, seed)
    assert int((batch.ops["flags"] & MT_F_REL1 != 0).sum()) > 100
    rc, exp = _oracle_doc(orc, batch, cap_props=1 << 15)
    assert rc == 0
    got = emu_huge_replay(batch, tiny_groups=tiny)
    assert int(got[0]["status"]) == 0, f"engine status {int(got[0]['status'])} at seq {int(got[0]['fail_seq'])}"
    assert compare_doc(exp, got) == []
    if n_ops >= 12000:
        assert int(got[0]["n_props"]) > 4096


@pytest.mark.parametrize("exact_tail,tiny", [(False, True), (True, False), (False, False)])
def test_huge_engine_annotate_adjust(orc, exact_tail, tiny):
    """Annotate-adjust in the huge tier (computePropertyValue, segmentPropertiesManager.ts:54-78, with
    the batch's number tables, adjust.h) and its PropertiesManager records: every document of the
    reference's conflict farms with adjusts, replayed by the emulated huge engine, equals the oracle
    (state and computed numbers), and its legacy summary from the engine's getAtSeq(minSeq) prop
    sets equals the oracle's SnapshotLegacy restatement."""
    from test_annotate_adjust import adjust_fixture_batch

    from fluidframework_amd import summary
    from mt_compare import emu_huge_replay_adjust
    batch, finals = adjust_fixture_batch(exact_tail)
    nums = []
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=4096, cap_chars=1 << 16, cap_props=4096,
                                                numbers=nums)
    assert rc == 0
    differs = 0
    for d in range(batch.n_docs):
        h, lv, ch, pr, legacy, got_nums = emu_huge_replay_adjust(batch, d, tiny_groups=tiny)
        assert int(h["status"]) == 0, (d, int(h["status"]), int(h["fail_seq"]))
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (h, lv, ch, pr)) == [], d
        assert np.array_equal(got_nums, nums[d]), d
        vals = summary.values_with_numbers(batch.values, got_nums)
        got = summary.legacy_summary(h, lv, ch, pr, batch.keys, vals, legacy_props=legacy)
        assert got == orc.mt_replay_summary(batch, d, batch.keys, batch.values), d
        differs += got != summary.legacy_summary(h, lv, ch, pr, batch.keys, vals)
    if not exact_tail:
        assert differs > 0
