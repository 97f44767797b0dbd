"""Sided obliterate (MergeTreeDeltaType.OBLITERATE_SIDED = 5, mergeTreeEnableSidedObliterate): the op's
pos1/pos2 are InteriorSequencePlaces {pos, before} (client.ts:680-700) replayed by
obliterateRangeSided (mergeTree.ts:2083-2260); packed with FMT_MT_F_START_BEFORE / FMT_MT_F_END_BEFORE.

Pins: a non-sided obliterate (pos1, pos2) IS obliterateRangeSided({pos1, Before}, {pos2 - 1, After})
(mergeTree.ts:2282-2286), so the 30 reference obliterate fixtures re-encoded as sided ops must still
reach every text checkpoint. Exclusive endpoints ({p, After} starts, {p, Before} ends) appear in no
reference fixture: those cases are parity unpinned (engine == oracle only).
"""
import numpy as np
import pytest

from test_obliterate import OB_FIXTURES

SIDED = 5
F_START_BEFORE, F_END_BEFORE = 8, 16
FMT_E_CAPACITY = -3


def as_sided(ops, rng=None):
    """Re-encode every non-sided obliterate as the equivalent sided op; with `rng`, then move about
    half of the endpoints to exclusive places: start {p, Before} -> {p - 1, After} (same boundary,
    reference on the previous character) and end {q, After} -> {q, Before} (the last character kept)."""
    ops = ops.copy()
    ob = ops["type"] == 4
    ops["pos2"][ob] -= 1
    ops["flags"][ob] |= F_START_BEFORE
    ops["type"][ob] = SIDED
    if rng is not None:
        idx = np.flatnonzero(ob)
        mv_start = idx[(rng.random(idx.size) < 0.5) & (ops["pos1"][idx] > 0)]
        ops["pos1"][mv_start] -= 1
        ops["flags"][mv_start] &= ~np.uint32(F_START_BEFORE)
        mv_end = idx[rng.random(idx.size) < 0.5]
        ops["flags"][mv_end] |= F_END_BEFORE
    return ops


def test_sided_encoding_counts():
    _, b, *_ = OB_FIXTURES[0]
    s = as_sided(b.ops)
    assert int((s["type"] == SIDED).sum()) == int((b.ops["type"] == 4).sum()) > 0
    assert not (s["type"] == 4).any()


@pytest.mark.parametrize("idx", range(0, len(OB_FIXTURES), 3), ids=[f[0] for f in OB_FIXTURES][::3])
def test_oracle_sided_encoding_reaches_fixture_checkpoints(orc, idx):
    name, batch, group_end, initial, results = OB_FIXTURES[idx]
    ops = as_sided(batch.ops)
    doc = orc.MergeTreeDoc()
    init = batch.doc_init[0]
    if init[1]:
        doc.insert_local(0, batch.text[init[0] : init[0] + init[1]].tobytes().decode("utf-16-le"))
    doc.start_collab(0)
    start = 0
    for g, end in enumerate(group_end):
        doc.apply(ops[start:end], batch.text, batch.props_off, batch.props_kv)
        assert doc.text() == results[g], f"group {g} result"
        start = end


def _sided_prefix(rng=None):
    from golden_data import prefix_batch

    batch, expected = prefix_batch(OB_FIXTURES[::3])
    batch.ops = as_sided(batch.ops, rng)
    return batch, expected


def _oracle_vs_emu(orc, batch):
    from mt_compare import compare_doc, emu_caps, emu_replay

    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    hdr, leaves, chars, props = emu_replay(batch)
    over = hdr["status"] == FMT_E_CAPACITY  # the runtime replays these again in the large tier
    for d in np.flatnonzero(~over):
        assert int(hdr[d]["status"]) == int(oh[d]["status"]), d
        if int(oh[d]["status"]) != 0:
            continue
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
    if over.any():
        cl, cc, cp = emu_caps(True)
        rc, oh2, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
        hdr, leaves, chars, props = emu_replay(batch, large=True)
        for d in np.flatnonzero(over):
            assert int(hdr[d]["status"]) == int(oh2[d]["status"]) == 0, d
            diffs = compare_doc((oh2[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
            assert not diffs, f"doc {d} (large tier): {diffs[:5]}"
    return oh


def test_emulated_engine_sided_encoding_matches_checkpoints(orc):
    from mt_compare import visible_text

    batch, expected = _sided_prefix()
    oh = _oracle_vs_emu(orc, batch)
    assert (oh["status"] == 0).all()
    from mt_compare import emu_replay

    hdr, leaves, chars, _ = emu_replay(batch)
    bad = [d for d, t in enumerate(expected) if visible_text(hdr[d], leaves[d], chars[d]) != t]
    assert not bad, bad[:5]


def test_emulated_engine_exclusive_endpoints_match_oracle(orc):
    """Parity unpinned: exclusive start/end places (no reference fixture holds one)."""
    batch, expected = _sided_prefix(np.random.default_rng(5))
    oh = _oracle_vs_emu(orc, batch)
    assert int((oh["status"] == 0).sum()) > batch.n_docs // 2
    # the exclusive places change some final texts (otherwise this test would pin nothing new)
    from mt_compare import emu_replay, visible_text

    hdr, leaves, chars, _ = emu_replay(batch)
    changed = sum(visible_text(hdr[d], leaves[d], chars[d]) != t for d, t in enumerate(expected) if hdr[d]["status"] == 0)
    assert changed > 0


def _replay_text(orc, msgs, initial="abcdef"):
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    sb = MergeTreeStreamBuilder()
    d = sb.begin_doc(initial)
    for m in msgs:
        d.add_message(m)
    batch = sb.finish()
    doc = orc.MergeTreeDoc()
    doc.insert_local(0, initial)
    doc.start_collab(0)
    doc.apply(batch.ops, batch.text, batch.props_off, batch.props_kv)
    return batch, doc.text()


def _msg(seq, ref, client, contents):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": 0, "contents": contents}


def test_host_packs_sided_places_and_exclusive_start_catches_concurrent_insert(orc):
    """{1, After}..{3, Before} removes only "c", but its start reference sits on "b", so a concurrent
    insert between "b" and "c" lies inside the obliterate and is obliterated on arrival
    (mergeTree.ts:1642-1746); the non-sided obliterate(2, 3) anchors on "c" and lets it stay."""
    ins = _msg(2, 0, "C", {"type": 0, "pos1": 2, "seg": "X"})
    sided = _msg(1, 0, "B", {"type": SIDED, "pos1": {"pos": 1, "before": False}, "pos2": {"pos": 3, "before": True}})
    batch, text = _replay_text(orc, [sided, ins])
    rec = batch.ops[0]
    assert (int(rec["type"]), int(rec["pos1"]), int(rec["pos2"])) == (SIDED, 1, 3)
    assert int(rec["flags"]) == F_END_BEFORE
    assert text == "abdef"
    _, text_ns = _replay_text(orc, [_msg(1, 0, "B", {"type": 4, "pos1": 2, "pos2": 3}), ins])
    assert text_ns == "abXdef"
    # a sided obliterate inside a GROUP keeps its side flags next to FMT_MT_F_GROUP_CONT
    grp = _msg(1, 0, "B", {"type": 3, "ops": [{"type": 1, "pos1": 0, "pos2": 1}, sided["contents"]]})
    batch, _ = _replay_text(orc, [grp])
    assert int(batch.ops[1]["flags"]) == F_END_BEFORE | 1


@pytest.mark.parametrize("rng_seed", [None, 5])
def test_emulated_engine_sided_catchup_ranges_match_oracle(orc, rng_seed):
    """Legacy catch-up ops (sequence.ts:395-452): a sided obliterate raises an OBLITERATE delta
    (mergeTree.ts:2249-2253), merged like the non-sided one; engine ranges == oracle ranges."""
    from fluidframework_amd import streams
    from mt_compare import emu_replay

    cap = 4096
    batch, _ = _sided_prefix(None if rng_seed is None else np.random.default_rng(rng_seed))
    streams.flag_catchup(batch.ops, batch.doc_op_offsets)
    rc, oh, *_rest, ocu = orc.mt_replay_batch(batch, cap_catchup=cap)
    eh, *_e, ecu = emu_replay(batch, cap_catchup=cap)
    checked = 0
    for d in range(batch.n_docs):
        if int(eh[d]["status"]) == FMT_E_CAPACITY:  # replayed in the large tier by the runtime
            continue
        n = int(oh[d]["n_catchup"])
        assert int(eh[d]["n_catchup"]) == n and np.array_equal(ecu[d][:n], ocu[d][:n]), d
        checked += int((ocu[d][:n]["type"] == 4).sum())
    assert checked > 0  # obliterate ranges were among those compared
