"""Legacy catch-up ops: regenerated contents of the messages a legacy SharedString
summary keeps after minSeq (sequence/src/sequence.ts:395-452, 949-1018; snapshotlegacy.ts:178-190).

No reference fixture pins a catch-up blob (the reference's legacyWithCatchUp snapshots are of
detached strings, whose catch-up list is empty), so parity is anchored three ways:
  - engine ranges == oracle ranges, bit-exact (emulated engine here, the GPU in -m gpu);
  - a size-independent property: loading the summary at minSeq and applying its catch-up messages
    (the way a client loads a legacy summary) reproduces the final text of the original replay;
  - the messages the reference's own fixtures hold keep every field and key order, with contents
    rewritten only where refSeq != seq - 1.
"""
import gzip
import json
import os

import numpy as np
import pytest

from fluidframework_amd import streams, summary, workloads
from fluidframework_amd.streams import MergeTreeStreamBuilder
from mt_compare import emu_replay

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "replay_msgs_0.40.json.gz")
CAP = 4096


def fixture_batch():
    fx = json.load(gzip.open(GOLDEN, "rt", encoding="utf-8"))
    b = MergeTreeStreamBuilder(keep_messages=True)
    finals = []
    for f in fx:
        g = f["groups"]
        d = b.begin_doc(g[0]["initialText"], observer="A")
        for gg in g:
            for m in gg["msgs"]:
                d.add_message(m)
        finals.append(g[-1]["resultText"])
    return b.finish(catchup=True), finals


def _text(h, leaves, chars):
    out = []
    for L in leaves[: int(h["n_leaves"])]:
        if int(L["rm_seq"]) == 0x7FFFFFFF and not int(L["pad"]) & 0x8000:  # (markers: no text)
            o, n = int(L["char_off"]), int(L["len"])
            out.append(chars[o : o + n].tobytes().decode("utf-16-le", "surrogatepass"))
    return "".join(out)


def reload_text(orc, h, leaves, chars, props, keys, values, msgs):
    """Text after loading the legacy summary at minSeq and applying its catch-up messages."""
    segs = summary.legacy_segments(h, leaves, chars, props, int(h["min_seq"]))
    b = MergeTreeStreamBuilder()
    d = b.begin_doc("".join(t for t, _, m in segs if not m), observer="observer")
    for m in msgs:
        d.add_message(m)
    rb = b.finish()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(rb)
    assert rc == 0
    return _text(oh[0], ol[0], oc[0])


def test_fixture_messages_are_flagged_by_window():
    batch, _ = fixture_batch()
    for d in range(batch.n_docs):
        a, b = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
        ops = batch.ops[a:b]
        msn = int(ops["min_seq"][-1])
        want = (ops["seq"] > msn) & (ops["ref_seq"] != ops["seq"] - 1)
        assert np.array_equal((ops["flags"] & streams.MT_F_CATCHUP) != 0, want)
        assert want.any()


def test_oracle_catchup_reload_reproduces_fixture_text(orc):
    batch, finals = fixture_batch()
    rc, h, l, c, p, _, cu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    assert rc == 0
    for d in range(batch.n_docs):
        msgs = summary.catchup_messages(batch.messages[d], cu[d][: h[d]["n_catchup"]], int(h[d]["min_seq"]))
        assert msgs and all(m["sequenceNumber"] > h[d]["min_seq"] for m in msgs)
        assert _text(h[d], l[d], c[d]) == finals[d]
        assert reload_text(orc, h[d], l[d], c[d], p[d], batch.keys, batch.values, msgs) == finals[d], d


def test_catchup_messages_keep_fields_and_order(orc):
    batch, _ = fixture_batch()
    rc, h, l, c, p, _, cu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    for d in range(batch.n_docs):
        min_seq = int(h[d]["min_seq"])
        msgs = summary.catchup_messages(batch.messages[d], cu[d][: h[d]["n_catchup"]], min_seq)
        orig = [m for m, _, _ in batch.messages[d] if m["sequenceNumber"] > min_seq]
        assert len(msgs) == len(orig)
        for got, src in zip(msgs, orig):
            assert list(got) == [k for k in src if k != "term"]  # spread keeps positions; term deleted
            assert got["minimumSequenceNumber"] == min_seq
            assert got["referenceSequenceNumber"] == got["sequenceNumber"] - 1
            if src["referenceSequenceNumber"] == src["sequenceNumber"] - 1:
                assert got["contents"] == src["contents"]
        blob = summary.catchup_blob(msgs)
        assert json.loads(blob) == msgs


@pytest.mark.parametrize("n_clients,seed", [(8, 3), (4, 11), (16, 5)])
def test_emulated_engine_catchup_matches_oracle_and_reloads(orc, n_clients, seed):
    batch = workloads.conflict_farm(24, n_clients=n_clients, ops_per_doc=1200, seed=seed)
    streams.flag_catchup(batch.ops, batch.doc_op_offsets)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    assert rc == 0
    eh, el, ec, ep, ecu = emu_replay(batch, cap_catchup=CAP)
    assert (eh["status"] == 0).all()
    for d in range(batch.n_docs):
        n = int(oh[d]["n_catchup"])
        assert n > 0 and int(eh[d]["n_catchup"]) == n
        assert np.array_equal(ecu[d][:n], ocu[d][:n]), d


def test_emulated_engine_catchup_on_fixtures(orc):
    batch, _ = fixture_batch()
    rc, oh, *_rest, ocu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    eh, el, ec, ep, ecu = emu_replay(batch, cap_catchup=CAP)
    for d in range(batch.n_docs):
        n = int(oh[d]["n_catchup"])
        assert int(eh[d]["n_catchup"]) == n and np.array_equal(ecu[d][:n], ocu[d][:n]), d


def test_catchup_capacity_overflow_is_reported(orc):
    batch, _ = fixture_batch()
    eh, *_rest = emu_replay(batch, cap_catchup=8)
    assert (eh["status"] == -3).all()  # FMT_E_CAPACITY, per document
