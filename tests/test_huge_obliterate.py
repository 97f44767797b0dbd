"""Obliterates in the huge tier (mergeTree.ts:515-635, 2083-2290; huge_engine.h
applyObliterate / obliterateOnInsert): the live-obliterate table (endpoint references as leaf id +
offset, ordinals = (group position, slot, index in block)), reference moves on splits and zamboni
appends, Obliterates.setMinSeq, and the obliterate-on-insert rule, as mt_engine.h has them.

Pins: the reference's 30 obliterate farms (merge-tree/src/test/results
`*-conflict-farm-with-obliterate-2.3.0.json`), replayed by the emulated huge engine with its index
invariants checked after every op, with normal and 16-slot groups, reach the fixtures' final text and
equal the oracle bit for bit; their sided re-encodings too (exclusive places: oracle only). Scaled
past the large tier (the farms on a 135,000-unit initial text), the runtime restarts them in the
huge tier on the GPU: engine == oracle.
"""
import numpy as np
import pytest

from mt_compare import compare_doc, emu_huge_replay, visible_text
from test_obliterate import OB_FIXTURES, long_obliterate_farms
from test_obliterate_sided import as_sided


def _oracle(orc, batch, doc=0):
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1024)
    assert rc == 0
    return oh[doc], ol[doc], oc[doc], op[doc]


@pytest.mark.parametrize("idx", range(len(OB_FIXTURES)), ids=[f[0] for f in OB_FIXTURES])
def test_emulated_huge_tier_obliterate_fixtures(orc, idx):
    name, batch, group_end, initial, results = OB_FIXTURES[idx]
    exp = _oracle(orc, batch)
    for tiny in (False, True):
        got = emu_huge_replay(batch, 0, tiny_groups=tiny)
        assert int(got[0]["status"]) == 0, (tiny, int(got[0]["status"]), int(got[0]["fail_seq"]))
        assert visible_text(got[0], got[1], got[2]) == results[-1], tiny
        assert compare_doc(exp, got) == [], tiny


@pytest.mark.parametrize("seed", [None, 5, 9])
def test_emulated_huge_tier_sided_obliterates(orc, seed):
    for name, batch, group_end, initial, results in OB_FIXTURES[::3]:
        from dataclasses import replace

        b = replace(batch, ops=as_sided(batch.ops, None if seed is None else np.random.default_rng(seed)))
        exp = _oracle(orc, b)
        got = emu_huge_replay(b, 0, tiny_groups=True)
        assert int(got[0]["status"]) == int(exp[0]["status"]) == 0, name
        if seed is None:
            assert visible_text(got[0], got[1], got[2]) == results[-1], name
        assert compare_doc(exp, got) == [], name


def _one(batch, d):
    from dataclasses import replace

    o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
    return replace(batch, ops=batch.ops[o0:o1], doc_op_offsets=np.array([0, o1 - o0], np.uint64),
                   doc_init=batch.doc_init[d : d + 1].copy())


@pytest.mark.parametrize("doc", [0, 3, 4, 5])
def test_emulated_huge_tier_scaled_obliterate_farm(orc, doc):
    """A farm on a 135,000-unit initial text (past the large tier): emulated huge engine == oracle.
    (Farms 3-5 keep appending short acked leaves onto the long initial run: zamboni recopies the run
    each time, which the merge area absorbs by compacting into its other half.)"""
    one = _one(long_obliterate_farms(extra=135000), doc)
    exp = _oracle(orc, one)
    got = emu_huge_replay(one, 0)
    assert int(got[0]["status"]) == 0 and int(got[0]["visible_len"]) > 131071
    assert compare_doc(exp, got) == []


def test_emulated_merge_area_compaction(orc, monkeypatch, capfd):
    """A merge area of 4x the document's text forces compactions: the state still == oracle."""
    import re

    one = _one(long_obliterate_farms(extra=135000), 3)
    exp = _oracle(orc, one)
    doc_chars = int(one.doc_init[0][1]) + int(one.ops["len"][one.ops["type"] == 0].sum())
    monkeypatch.setenv("FMT_EMU_TEXTCAP", str(len(one.text) + 4 * doc_chars + 64))
    got = emu_huge_replay(one, 0)
    n = int(re.search(r"compactions (\d+)", capfd.readouterr().err).group(1))
    assert n >= 3
    assert int(got[0]["status"]) == 0
    assert compare_doc(exp, got) == []


@pytest.mark.gpu
def test_scaled_obliterate_farms_restart_in_huge_tier_on_gpu(orc):
    """The 30 obliterate farms on 135,000-unit initial texts: the large tier reports FMT_E_CAPACITY and
    the runtime replays them in the huge tier — engine == oracle for every document."""
    from fluidframework_amd import native

    batch = long_obliterate_farms(extra=135000)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1024)
    assert rc == 0
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        assert (hdrs["status"] == 0).all()
        for d in range(batch.n_docs):
            assert int(hdrs[d]["visible_len"]) > 131071
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)), d
    finally:
        eng.close()
