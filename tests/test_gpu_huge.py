"""T3 on the GPU (BASELINE config 5): documents beyond the large tier are replayed by the huge-document
engine (csrc/huge_engine.h, hugedoc.hip) through the same C ABI, bit-exact against the oracle (with
its remote-length index): every leaf field, the text, the prop sets, the header."""
import copy

import numpy as np
import pytest

from fluidframework_amd import native, workloads
from mt_compare import compare_doc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = native.Engine(0)
    yield e
    e.close()


def _oracle(orc, batch, doc=0, cap_props=4096):
    orc.set_index(True)
    try:
        sub = _one_doc(batch, doc)
        sd = sub.snapshots[0] if sub.snapshots is not None else None
        segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None and sd["loaded"] else 0
        nops = len(sub.ops)
        rc, h, lv, ch, pr, *_ = orc.mt_replay_timed(sub, 0, 0, cap_leaves=segs + 3 * nops + 4096,
                                                    cap_chars=len(sub.text) + 8, cap_props=cap_props)
    finally:
        orc.set_index(False)
    return rc, (h, lv[: int(h["n_leaves"])], ch[: int(h["n_chars"])], pr[: int(h["n_props"])])


def _one_doc(batch, d):
    b = copy.copy(batch)
    o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
    b.ops = batch.ops[o0:o1]
    b.doc_op_offsets = np.array([0, o1 - o0], dtype=np.uint64)
    b.doc_init = batch.doc_init[d : d + 1]
    if batch.snapshots is not None:
        b.snapshots = batch.snapshots[d : d + 1]
    return b


def _concat(batches):
    """One batch holding every document of `batches` (same props table: conflict farm and T3 share it)."""
    from fluidframework_amd.streams import SNAPSHOT_DOC_DTYPE, SNAPSHOT_SEG_DTYPE

    ops, offs, texts, init, snaps, segs = [], [0], [], [], [], []
    tbase, sbase = 0, 0
    for b in batches:
        o = b.ops.copy()
        o["payload"][o["type"] == 0] += tbase
        ops.append(o)
        offs.extend((np.asarray(b.doc_op_offsets[1:], dtype=np.int64) + offs[-1]).tolist())
        texts.append(b.text)
        di = b.doc_init.copy()
        di[:, 0] += tbase
        init.append(di)
        if b.snapshots is not None:
            sd = b.snapshots.copy()
            sd["first_seg"] += sbase
            sg = b.snapshot_segs.copy()
            sg["text"] += tbase
            snaps.append(sd)
            segs.append(sg)
            sbase += len(sg)
        else:
            snaps.append(np.zeros(b.n_docs, dtype=SNAPSHOT_DOC_DTYPE))
        tbase += len(b.text)
    first = batches[0]
    return first.__class__(
        ops=np.concatenate(ops), doc_op_offsets=np.asarray(offs, dtype=np.uint64), text=np.concatenate(texts),
        doc_init=np.concatenate(init), props_off=first.props_off, props_kv=first.props_kv, keys=first.keys,
        values=first.values, snapshots=np.concatenate(snaps),
        snapshot_segs=np.concatenate(segs) if segs else np.zeros(0, dtype=SNAPSHOT_SEG_DTYPE))


@pytest.mark.parametrize("segs,ops,clients,lag,rng,seed", [
    (5000, 8000, 63, 4096, 8, 3),
    (60000, 40000, 63, 4096, 8, 4),
    (30000, 20000, 16, 1000, 300, 5),
])
def test_huge_doc_matches_oracle(orc, engine, segs, ops, clients, lag, rng, seed):
    batch = workloads.t3_stream(segs, ops, n_clients=clients, max_lag=lag, max_range=rng, seed=seed)
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []


def test_mixed_batch_small_large_and_huge_documents(orc, engine):
    """Huge documents replay beside ordinary ones (small tier) in one fmt_mt_run."""
    farm = workloads.conflict_farm(24, n_clients=8, ops_per_doc=600, seed=8)
    t3a = workloads.t3_stream(3000, 4000, n_clients=31, max_lag=700, seed=9)
    t3b = workloads.t3_stream(9000, 6000, n_clients=63, max_lag=4096, max_range=20, seed=10)
    batch = _concat([farm, t3a, farm, t3b])
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert (hdrs["status"] == 0).all()
    for d in range(batch.n_docs):
        rc, exp = _oracle(orc, batch, d)
        assert rc == 0
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert compare_doc(exp, (hdrs[d], lv, ch, pr)) == [], d
    engine.mt_run()  # a second run over the same state replays from the inputs again
    assert np.array_equal(engine.mt_headers(), hdrs)


def test_t3_million_segments(orc, engine):
    batch = workloads.t3_stream(1_000_000, 100_000, n_clients=63, max_lag=4096, seed=12)
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []


def test_t3_ten_million_segments_digest(orc, engine):
    """T3 at its full document size (BASELINE config 5: 10M segments loaded from a legacy summary's
    header + body, as bench.py loads it; 63 writers, refSeq lag up to 4096) over a 2e5-op slice: the
    whole document's state digest (every leaf field, props by value, text, header;
    fmt_mt_state_digest) equals the oracle's digest of its own replay. The full 1e7-op
    run is bench.py --workload t3 --t3-check."""
    batch = workloads.as_legacy_load(workloads.t3_stream(10_000_000, 200_000, n_clients=63, max_lag=4096, seed=14))
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    got = engine.mt_digests()
    orc.set_index(True)  # (the oracle's remote-length index: the T3 CPU baseline's own configuration)
    try:
        rc, exp, st, _ = orc.mt_replay_digest(batch, 0, 1, threads=1)
    finally:
        orc.set_index(False)
    assert rc == 0 and int(st[0]) == 0
    assert int(got[0]) == int(exp[0])


def test_huge_inserts_with_props(orc, engine):
    """seg {text, props} inserts in a huge document (prop sets interned up to 4096)."""
    batch = workloads.with_insert_props(workloads.t3_stream(200_000, 30_000, n_clients=32, max_lag=1024, max_range=8, seed=23))
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    leaves, chars, props = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], leaves, chars, props)) == []


def test_huge_loaded_markers(orc, engine):
    """Marker segments in a huge document's summary (every third 1-unit spec) on the GPU."""
    import dataclasses

    from fluidframework_amd.streams import MT_SEG_MARKER
    batch = workloads.t3_stream(200_000, 20_000, n_clients=16, max_lag=512, max_range=8, seed=31)
    segs = batch.snapshot_segs.copy()
    idx = np.nonzero(segs["len"] == 1)[0][::3]
    segs["len"][idx] = 1 | MT_SEG_MARKER
    batch = dataclasses.replace(batch, snapshot_segs=segs)
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    leaves, chars, props = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], leaves, chars, props)) == []


def test_unsupported_huge_document_fails_alone(orc, engine):
    """A summary-loaded document past the large tier that asks for something the huge tier does not
    replay (here a writer with short id 255: the huge tier keeps ids up to 253) fails alone, with
    FMT_E_UNSUPPORTED in its own header; one holding a loader segment (FMT_MT_F_LOADSEG, which the
    huge tier replays since round 5) equals the oracle; the ordinary and huge documents beside them
    replay as in a batch without them."""
    import dataclasses

    from fluidframework_amd.streams import MT_F_LOADSEG, NON_COLLAB_CLIENT, SNAPSHOT_INFO_DTYPE, STAMP_DTYPE
    farm = workloads.conflict_farm(24, n_clients=8, ops_per_doc=600, seed=8)
    t3a = workloads.t3_stream(3000, 4000, n_clients=31, max_lag=700, seed=9)
    ld = workloads.t3_stream(9000, 6000, n_clients=63, max_lag=4096, max_range=20, seed=10)
    bad = workloads.t3_stream(9000, 6000, n_clients=63, max_lag=4096, max_range=20, seed=11)
    batch = _concat([farm, t3a, ld, bad, farm])
    info = np.zeros(len(batch.snapshot_segs), dtype=SNAPSHOT_INFO_DTYPE)
    info["ins_client"] = NON_COLLAB_CLIENT  # (rows without merge info: the loads are unchanged)
    ops = batch.ops.copy()
    o0 = int(batch.doc_op_offsets[farm.n_docs + 1])
    first_insert = o0 + int(np.nonzero(ld.ops["type"] == 0)[0][0])
    ops["flags"][first_insert] |= MT_F_LOADSEG
    ops["pos1"][first_insert] = 0  # (merge-info row 0)
    o1 = int(batch.doc_op_offsets[farm.n_docs + 2])
    ops["client"][o1 + 10] = 255  # (a writer past the huge tier's 253; 254 names NonCollab)
    batch = dataclasses.replace(batch, ops=ops, snapshot_info=info, snapshot_stamps=np.zeros(1, dtype=STAMP_DTYPE))
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers(raise_on_failed_docs=False)
    bad_doc = farm.n_docs + 2
    assert int(hdrs[bad_doc]["status"]) == native.FMT_E_UNSUPPORTED
    for d in range(batch.n_docs):
        if d == bad_doc:
            continue
        rc, exp = _oracle(orc, batch, d)
        assert int(hdrs[d]["status"]) == int(exp[0]["status"]), d
        if rc == 0:
            lv, ch, pr = engine.mt_doc(d, hdrs[d])
            assert compare_doc(exp, (hdrs[d], lv, ch, pr)) == [], d


@pytest.mark.parametrize("n_ops,seed", [(6000, 5), (9000, 6)])
def test_huge_annotate_adjust_on_gpu(orc, engine, n_ops, seed):
    """Annotate-adjust in documents past the large tier (grown from their start: marker-rich streams
    whose annotates adjust "weight"): state, computed numbers and the legacy summary with
    getAtSeq(minSeq) props (the huge tier's PropertiesManager records) == oracle."""
    from marker_docs import marker_batch

    from fluidframework_amd.summary import legacy_summary, values_with_numbers
    batch = marker_batch(1, n_ops, seed=seed, adjust=True)
    assert batch.adjusts is not None
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    assert int(hdrs[0]["n_leaves"]) > 2048  # (past the large tier)
    nums = []
    orc.set_index(True)
    try:
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=4 * n_ops + 64, cap_chars=len(batch.text) + 8,
                                                    cap_props=1 << 15, numbers=nums)
    finally:
        orc.set_index(False)
    assert rc == 0
    exp = (oh[0], ol[0][: int(oh[0]["n_leaves"])], oc[0][: int(oh[0]["n_chars"])], op[0][: int(oh[0]["n_props"])])
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
    got_nums = engine.mt_numbers(0)
    assert np.array_equal(got_nums, nums[0])
    want = orc.mt_replay_summary(batch, 0, batch.keys, batch.values)
    engine.mt_summarize_legacy(batch.keys, batch.values)
    assert engine.mt_summary(0) == want
    vals = values_with_numbers(batch.values, got_nums)
    assert legacy_summary(hdrs[0], lv, ch, pr, batch.keys, vals, legacy_props=engine.mt_legacy_props(0, hdrs[0])) == want


@pytest.mark.parametrize("n_ops,split,seed", [(6000, 0, 2), (12000, 9000, 4)])
def test_huge_relative_positions_on_gpu(orc, engine, n_ops, split, seed):
    """Legacy relativePos1 inserts in documents past the large tier: one grown from its start (the
    large tier runs out of leaves and prop sets), one loaded from a summary holding its first
    `split` messages' Markers; == oracle."""
    from marker_docs import marker_batch
    from test_huge_emulated import marker_reload
    batch = marker_batch(1, n_ops, seed=seed) if split == 0 else marker_reload(orc, n_ops, split, seed)
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    assert int(hdrs[0]["n_leaves"]) > 2048  # (past the large tier)
    rc, exp = _oracle(orc, batch, cap_props=1 << 15)
    assert rc == 0
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
    # the bulk legacy summary (summaryRunsKernel with the engine's match classes: > 4096 prop sets)
    engine.mt_summarize_legacy(batch.keys, batch.values)
    assert engine.mt_summary(0) == orc.mt_replay_summary(batch, 0, batch.keys, batch.values)
    if split:
        assert int(hdrs[0]["n_props"]) > 4096


@pytest.mark.parametrize("segs,ops,props_every,seed", [
    (30000, 20000, 0, 21),
    (1_000_000, 100_000, 5, 22),
])
def test_huge_legacy_header_and_body_on_gpu(orc, engine, segs, ops, props_every, seed):
    """T3 from a summary in SnapshotLegacy.emit's shape (header chunk ~10,000 units, body chunk
    appended by loadBody) with props on some segment specs == oracle on the GPU."""
    batch = workloads.as_legacy_load(workloads.t3_stream(segs, ops, n_clients=63, max_lag=4096, seed=seed),
                                     props_every=props_every)
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []


def test_huge_zamboni_empties_the_root_on_gpu(orc, engine):
    batch = workloads.emptying_stream(3000, 600, seed=4)
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []


def test_huge_legacy_summary_with_catchup_on_gpu(orc, engine):
    """The whole legacy summary of a huge document loaded from a SnapshotLegacy-shaped summary —
    header and body blobs at its minSeq plus the catchupOps blob regenerated from the catch-up
    ranges the huge engine records (sequence.ts:949-1018, snapshotlegacy.ts:126-193) — equals the
    one built from the oracle's state and ranges."""
    from fluidframework_amd import summary
    from fluidframework_amd.streams import MT_F_CATCHUP, flag_catchup, op_messages
    from fluidframework_amd.summary import legacy_summary
    batch = workloads.as_legacy_load(workloads.t3_stream(60000, 30000, n_clients=63, max_lag=4096, max_range=40, seed=27),
                                     props_every=6)
    flag_catchup(batch.ops, batch.doc_op_offsets)
    n_flag = int(((batch.ops["flags"] & MT_F_CATCHUP) != 0).sum())
    assert n_flag > 1000
    cap = 16 * n_flag + 16
    n_segs = int(batch.snapshots[0]["n_header"]) + int(batch.snapshots[0]["n_body"])
    orc.set_index(True)
    try:
        rc, oh, olv, och, opr, _, ocu = orc.mt_replay_batch(batch, cap_leaves=n_segs + 3 * len(batch.ops) + 8,
                                                           cap_chars=len(batch.text) + 8, cap_props=4096, cap_catchup=cap)
    finally:
        orc.set_index(False)
    assert rc == 0
    h = oh[0]
    exp = (h, olv[0][: int(h["n_leaves"])], och[0][: int(h["n_chars"])], opr[0][: int(h["n_props"])])
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
    cu = engine.mt_catchup(0, hdrs[0])
    assert np.array_equal(cu, ocu[0][: int(h["n_catchup"])])
    engine.mt_summarize_legacy(batch.keys, batch.values)
    names = [f"client-{k}" for k in range(64)]
    msgs = op_messages(batch, 0, int(h["min_seq"]), names)
    got = (*engine.mt_summary(0), summary.catchup_blob(summary.catchup_messages(msgs, cu, int(hdrs[0]["min_seq"]))))
    want = (*legacy_summary(*exp, batch.keys, batch.values),
            summary.catchup_blob(summary.catchup_messages(msgs, ocu[0][: int(h["n_catchup"])], int(h["min_seq"]))))
    assert got == want
    assert got[1] is not None and got[2] is not None


def test_huge_remove_order_on_gpu(orc, engine):
    """SnapshotV1 remove order from a huge document (header + body summary, overlapping removes of
    lagging writers): each leaf's remove stamps == the oracle's, and its V1 summary from GPU state ==
    the one from the oracle's stamp lists."""
    from fluidframework_amd import summary
    from fluidframework_amd.streams import flag_remove_order
    batch = workloads.as_legacy_load(workloads.t3_stream(40000, 20000, n_clients=63, max_lag=2000, max_range=60, seed=43))
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
    rm = engine.mt_remove_order(0, hdrs[0])
    assert len(rm) > 0
    want = orc.mt_removers(batch, 0)
    got = summary.removers_from_engine(lv, int(hdrs[0]["n_leaves"]), rm, batch.ops)
    ms, multi = int(hdrs[0]["min_seq"]), 0
    for i in range(int(hdrs[0]["n_leaves"])):
        r = int(lv[i]["rm_seq"])
        if r != summary.NOT_REMOVED and r > ms:
            assert got.get(i) == want.get(i), i
            multi += len(want[i]) > 1
    assert multi > 0
    names = [f"client-{k}" for k in range(64)]
    assert summary.v1_summary(hdrs[0], lv, ch, pr, batch.keys, batch.values, names, got) == \
        summary.v1_summary(hdrs[0], lv, ch, pr, batch.keys, batch.values, names, want)


def test_huge_v1_merge_info_load_on_gpu(orc, engine):
    """A huge document loaded from a SnapshotV1 summary whose header segments carry merge info above
    minSeq (inserted by writers, removed by one to three of them): == oracle on the GPU."""
    from v1_huge import with_v1_merge_info
    batch = with_v1_merge_info(workloads.t3_stream(30000, 20000, n_clients=31, max_lag=800, max_range=8, seed=52))
    rc, exp = _oracle(orc, batch)
    assert rc == 0
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert int(hdrs[0]["status"]) == 0, (int(hdrs[0]["status"]), int(hdrs[0]["fail_seq"]))
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert compare_doc(exp, (hdrs[0], lv, ch, pr)) == []
