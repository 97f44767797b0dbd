"""Loading a legacy SharedString summary into engine state.

SnapshotLoader (merge-tree/src/snapshotLoader.ts:59-348) + reloadFromSegments (mergeTree.ts:751-800)
+ SharedSegmentSequence.loadCore's catch-up replay (sequence/src/sequence.ts:818-863).

Pinned by the reference's own legacy snapshot fixtures: loading each and summarizing again gives
the fixture's blobs byte for byte (oracle, and the engine's large tier: these documents overflow
the small tier's 512 leaves / 2048 UTF-16 units). Then, on the reference's replay fixture messages and on generated conflict farms:
  - the engine (emulated here, the GPU in -m gpu) equals the oracle bit for bit after a load;
  - summary → load (+ catch-up ops) → summary is a fixed point, and the loaded document's text after
    its catch-up ops equals the original replay's final text.
"""
import numpy as np
import pytest

from fluidframework_amd import native, summary, workloads
from fluidframework_amd.streams import MergeTreeStreamBuilder
from golden_data import snapshot_trees
from mt_compare import compare_doc, emu_caps, emu_replay
from test_catchup import CAP, _text, fixture_batch
from test_oracle_golden import _blobs

CHUNK = 40  # small first chunk so that short documents get a body chunk too


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"])
def test_oracle_load_resummarize_reference_snapshot(orc, name):
    blobs = _blobs(snapshot_trees()[name])
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(blobs["header"], blobs.get("body"))
    batch = b.finish()
    rc, h, l, c, p, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 20, cap_props=1024)
    assert rc == 0
    head, body = summary.legacy_summary(h[0], l[0], c[0], p[0], batch.keys, batch.values)
    assert head == blobs["header"] and body == blobs.get("body")


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"])
def test_large_tier_loads_reference_snapshot(orc, name):
    """The reference snapshots (8.9k-89k chars, up to 1112 segments) overflow the small tier and load
    in the large tier (emulated here; on the GPU the runtime escalates them by itself): engine ==
    oracle, and summarizing again gives the fixture's blobs byte for byte."""
    blobs = _blobs(snapshot_trees()[name])
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(blobs["header"], blobs.get("body"))
    batch = b.finish()
    assert emu_replay(batch)[0][0]["status"] == native.FMT_E_CAPACITY
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    eh, el, ec, ep = emu_replay(batch, large=True)
    assert eh[0]["status"] == 0
    assert not compare_doc((oh[0], ol[0], oc[0], op[0]), (eh[0], el[0], ec[0], ep[0]))
    head, body = summary.legacy_summary(eh[0], el[0], ec[0], ep[0], batch.keys, batch.values)
    assert head == blobs["header"] and body == blobs.get("body")


def summaries_of(orc, batch, chunk=CHUNK, catchup=True):
    rc, h, l, c, p, _, cu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    assert rc == 0
    out = []
    for d in range(batch.n_docs):
        head, body = summary.legacy_summary(h[d], l[d], c[d], p[d], batch.keys, batch.values, chunk_size=chunk)
        blob = None
        if catchup and batch.messages:
            blob = summary.catchup_blob(summary.catchup_messages(batch.messages[d], cu[d][: h[d]["n_catchup"]],
                                                                int(h[d]["min_seq"])))
        out.append((head, body, blob, _text(h[d], l[d], c[d])))
    return out


def _minseq_text(head, body):
    import json

    segs = json.loads(head)["segmentTexts"] + (json.loads(body)["segmentTexts"] if body else [])
    return "".join(x if isinstance(x, str) else x["text"] for x in segs)


def reload_batch(sums, keep_messages=True):
    b = MergeTreeStreamBuilder(keep_messages=keep_messages)
    for head, body, blob, _ in sums:
        b.begin_doc_from_summary(head, body, blob)
    return b.finish(catchup=keep_messages)


def test_load_fixture_summaries_fixed_point_and_text(orc):
    batch, finals = fixture_batch()
    sums = summaries_of(orc, batch)
    assert any(s[1] is not None for s in sums)  # the body path is exercised
    rb = reload_batch(sums)
    again = summaries_of(orc, rb)
    for d, (s0, s1) in enumerate(zip(sums, again)):
        assert s1[3] == finals[d], d                    # loaded + catch-up ops = final text
        assert s1[2] == s0[2], d                        # the catch-up blob is a fixed point
        # The minSeq text is a fixed point too. The props are not, in the reference either: the
        # legacy summary writes each segment's *current* props (PropertiesManager.getAtSeq only
        # rolls back adjusts, segmentPropertiesManager.ts:328-344) while catch-up annotates skip
        # segments removed meanwhile (sequence.ts:395-452 sees only deltaSegments), so an earlier
        # catch-up annotate can overwrite a later value on a segment present at minSeq.
        assert _minseq_text(s1[0], s1[1]) == _minseq_text(s0[0], s0[1]), d


def test_emulated_engine_matches_oracle_after_load(orc):
    batch, _ = fixture_batch()
    rb = reload_batch(summaries_of(orc, batch))
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(rb, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    eh, el, ec, ep = emu_replay(rb)
    for d in range(rb.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


@pytest.mark.parametrize("seed", [4, 9])
def test_emulated_engine_load_conflict_farm_summaries(orc, seed):
    cf = workloads.conflict_farm(40, n_clients=8, ops_per_doc=1200, seed=seed)
    sums = summaries_of(orc, cf, chunk=60, catchup=False)
    rb = reload_batch(sums, keep_messages=False)
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(rb, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    eh, el, ec, ep = emu_replay(rb)
    for d in range(rb.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
        head, body = summary.legacy_summary(eh[d], el[d], ec[d], ep[d], rb.keys, rb.values, chunk_size=60)
        assert (head, body) == sums[d][:2], d


def test_invalid_catchup_ops_are_rejected():
    batch, _ = fixture_batch()
    import json

    head = json.dumps({"chunkStartSegmentIndex": 0, "chunkSegmentCount": 1, "chunkLengthChars": 1,
                       "totalLengthChars": 1, "totalSegmentCount": 1, "chunkSequenceNumber": 10,
                       "segmentTexts": ["a"], "headerMetadata": {"orderedChunkMetadata": [{"id": "header"}],
                                                                 "sequenceNumber": 10, "totalLength": 1,
                                                                 "totalSegmentCount": 1}})
    bad = json.dumps([{"clientId": "B", "sequenceNumber": 9, "referenceSequenceNumber": 9,
                       "minimumSequenceNumber": 10, "contents": {"pos1": 0, "seg": "x", "type": 0}}])
    with pytest.raises(ValueError, match="Invalid catchup"):
        MergeTreeStreamBuilder().begin_doc_from_summary(head, None, bad)


def test_snapshot_layouts():
    from fluidframework_amd.streams import SNAPSHOT_DOC_DTYPE, SNAPSHOT_SEG_DTYPE

    assert SNAPSHOT_DOC_DTYPE.itemsize == 32 and SNAPSHOT_SEG_DTYPE.itemsize == 12
    assert native.LEAF_DTYPE.itemsize == 32
