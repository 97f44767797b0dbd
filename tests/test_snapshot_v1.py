"""SharedString SnapshotV1 summaries (merge-tree/src/snapshotV1.ts:90-265,
snapshotChunks.ts:141-180, chosen by newMergeTreeSnapshotFormat in Client.summarize, client.ts:1569).

Pinned by the reference's own v1 fixtures (sequence/src/test/snapshots/v1/*.json, committed under
tests/golden/snapshots_v1.json): each loads (V1 chunks, or the legacy fixture of the same string) and
summarizes again to the fixture's blobs byte for byte — oracle and the engine's large tier.

Merge info (seq/client above minSeq, removedSeq/removedClient/removedClientIds) appears only for
collaborative documents, which no reference fixture holds: that part is pinned by the oracle only
(it keeps every remove stamp in order, stamps.ts:144-158). The engine's remove-order slab
(FMT_MT_F_RMORDER) plus the first remover's op give the same ordered lists and the same bytes.
"""
import json

import numpy as np
import pytest

from fluidframework_amd import summary
from fluidframework_amd.streams import MergeTreeStreamBuilder, UnsupportedOp, flag_remove_order
from golden_data import snapshot_trees
from mt_compare import compare_doc, emu_caps, emu_replay, visible_text
from test_catchup import fixture_batch

NAMES = ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"]


def _v1_blobs(tree):
    assert [e["path"] for e in tree["entries"]] == ["content"]
    content = {e["path"]: e["value"]["contents"] for e in tree["entries"][0]["value"]["entries"]}
    bodies = [content[f"body_{k}"] for k in range(len(content) - 1)]
    assert set(content) == {"header", *[f"body_{k}" for k in range(len(bodies))]}
    return content["header"], bodies


def _load_v1(name):
    head, bodies = _v1_blobs(snapshot_trees("v1")[name])
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(head, bodies)
    return b.finish(), head, bodies


@pytest.mark.parametrize("name", NAMES)
def test_oracle_v1_fixture_round_trip(orc, name):
    batch, head, bodies = _load_v1(name)
    rc, h, l, c, p, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 20, cap_props=1024)
    assert rc == 0
    got = summary.v1_summary(h[0], l[0], c[0], p[0], batch.keys, batch.values, batch.clients[0], {})
    assert got == (head, bodies)


@pytest.mark.parametrize("name", NAMES)
def test_legacy_fixture_resummarizes_as_v1_fixture(orc, name):
    """The legacy and v1 fixtures are the same strings: load legacy, emit V1, get the v1 fixture."""
    from test_oracle_golden import _blobs

    blobs = _blobs(snapshot_trees()[name])
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(blobs["header"], blobs.get("body"))
    batch = b.finish()
    rc, h, l, c, p, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 20, cap_props=1024)
    assert rc == 0
    _, head, bodies = _load_v1(name)
    assert summary.v1_summary(h[0], l[0], c[0], p[0], batch.keys, batch.values, batch.clients[0], {}) == (head, bodies)


@pytest.mark.parametrize("name", NAMES)
def test_engine_large_tier_v1_fixture_round_trip(name):
    batch, head, bodies = _load_v1(name)
    eh, el, ec, ep = emu_replay(batch, large=True)
    assert eh[0]["status"] == 0
    assert summary.v1_summary(eh[0], el[0], ec[0], ep[0], batch.keys, batch.values, batch.clients[0], {}) == (head, bodies)


def test_v1_merge_info_segments_load_with_their_stamps():
    """specToSegment (snapshotLoader.ts:105-175): the insert stamp from seq/client; setRemove stamps
    at removedSeq for every removedClientIds entry (removedClient alone in the back-compat format);
    sliceRemove stamps from movedSeqs/movedClientIds; all sorted by seq."""
    segs = [{"json": "a", "seq": 3, "client": "B"},
            {"json": "bc", "removedSeq": 4, "removedClient": "C"},
            {"json": "d", "seq": 2, "client": "C", "removedSeq": 5, "removedClient": "B", "removedClientIds": ["B", "D"],
             "movedSeq": 4, "movedSeqs": [4, 6], "movedClientIds": ["D", "B"]}]
    head = json.dumps({"version": "1", "segmentCount": 3, "length": 4, "segments": segs, "startIndex": 0,
                       "headerMetadata": {"minSequenceNumber": 1, "sequenceNumber": 6,
                                          "orderedChunkMetadata": [{"id": "header"}], "totalLength": 4,
                                          "totalSegmentCount": 3}})
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(head, [])
    batch = b.finish()
    assert batch.clients[0] == ["snapshot", "B", "C", "D"]
    info = [tuple(int(x) for x in r) for r in batch.snapshot_info]
    assert info == [(3, 1, 0, 0), (0, -2, 0, 1), (2, 2, 1, 4)]
    st = [tuple(int(x) for x in r)[:3] for r in batch.snapshot_stamps]
    assert st == [(4, 2, 0), (4, 3, 1), (5, 1, 0), (5, 3, 0), (6, 1, 1)]


def _collab_batch():
    batch, _ = fixture_batch()
    batch.ops["flags"] &= ~np.uint32(2)  # no catch-up recording (FMT_MT_F_CATCHUP) here
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    return batch


def _doc_ops(batch, d):
    return batch.ops[int(batch.doc_op_offsets[d]) : int(batch.doc_op_offsets[d + 1])]


def test_engine_remove_order_matches_oracle_stamps():
    """Engine (emulated) remove order == the oracle's remove stamp lists for every leaf removed above
    minSeq; V1 summaries with merge info are byte-identical."""
    import oracle as orc

    batch = _collab_batch()
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    eh, el, ec, ep, erm = emu_replay(batch, cap_rm=8192)
    multi = 0
    for d in range(batch.n_docs):
        assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d]))
        want = orc.mt_removers(batch, d)
        got = summary.removers_from_engine(el[d], int(eh[d]["n_leaves"]), erm[d][: eh[d]["n_rm_order"]],
                                           _doc_ops(batch, d))
        ms = int(eh[d]["min_seq"])
        for i in range(int(eh[d]["n_leaves"])):
            rm = int(el[d][i]["rm_seq"])
            if rm != summary.NOT_REMOVED and rm > ms:
                assert got.get(i) == want.get(i), (d, i)
                multi += len(want[i]) > 1
        v_or = summary.v1_summary(oh[d], ol[d], oc[d], op[d], batch.keys, batch.values, batch.clients[d], want)
        v_en = summary.v1_summary(eh[d], el[d], ec[d], ep[d], batch.keys, batch.values, batch.clients[d], got)
        assert v_or == v_en, d
    assert multi > 0  # overlapping removes (more than one removedClientId) are exercised


def test_v1_merge_info_shape():
    """Segments above minSeq carry seq/client, removed ones removedSeq/removedClient/removedClientIds,
    in the key order SnapshotV1.extractSync assigns them (snapshotV1.ts:226-250)."""
    import json

    import oracle as orc

    batch = _collab_batch()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    seen_removed = seen_ins = 0
    for d in range(batch.n_docs):
        head, bodies = summary.v1_summary(oh[d], ol[d], oc[d], op[d], batch.keys, batch.values, batch.clients[d],
                                          orc.mt_removers(batch, d))
        segs = [s for blob in [head] + bodies for s in json.loads(blob)["segments"]]
        for s in segs:
            if isinstance(s, dict) and "json" in s:
                keys = list(s)
                assert keys[0] == "json"
                if "seq" in s:
                    seen_ins += 1
                    assert keys[1:3] == ["seq", "client"] and s["seq"] > oh[d]["min_seq"]
                if "removedSeq" in s:
                    seen_removed += 1
                    assert keys[-3:] == ["removedSeq", "removedClient", "removedClientIds"]
                    assert s["removedClient"] == s["removedClientIds"][0]
        meta = json.loads(head)["headerMetadata"]
        assert meta["minSequenceNumber"] == oh[d]["min_seq"] and meta["sequenceNumber"] == oh[d]["cur_seq"]
        assert [m["id"] for m in meta["orderedChunkMetadata"]] == ["header"] + [f"body_{k}" for k in range(len(bodies))]
    assert seen_removed > 0 and seen_ins > 0


def test_engine_remove_order_matches_oracle_on_conflict_farm():
    import oracle as orc
    from fluidframework_amd import workloads

    batch = workloads.conflict_farm(24, n_clients=8, ops_per_doc=1000, seed=31)
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    eh, el, ec, ep, erm = emu_replay(batch, cap_rm=1 << 14)
    assert (eh["status"] == 0).all()
    multi = 0
    for d in range(batch.n_docs):
        want = orc.mt_removers(batch, d)
        got = summary.removers_from_engine(el[d], int(eh[d]["n_leaves"]), erm[d][: eh[d]["n_rm_order"]],
                                           _doc_ops(batch, d))
        ms = int(eh[d]["min_seq"])
        for i in range(int(eh[d]["n_leaves"])):
            rm = int(el[d][i]["rm_seq"])
            if rm != summary.NOT_REMOVED and rm > ms:
                assert got.get(i) == want.get(i), (d, i)
                multi += len(want[i]) > 2
    assert multi > 0  # three or more removers: the order the remove-client mask cannot give


def obliterate_v1_batch(stride=8):
    """The reference's obliterate conflict-farm fixtures (2.3.0), one document per 8th text
    checkpoint (the fixtures' last checkpoint included), flagged for SnapshotV1 merge info."""
    from dataclasses import replace

    from golden_data import prefix_batch, replay_fixtures

    batch, _ = prefix_batch(list(replay_fixtures("replay_obliterate_2.3.0.npz")))
    keep = [d for d in range(batch.n_docs) if d % stride == stride - 1]
    offs, ops, init = [0], [], []
    for d in keep:
        a, b = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
        ops.append(batch.ops[a:b])
        offs.append(offs[-1] + (b - a))
        init.append(batch.doc_init[d])
    sub = replace(batch, ops=np.concatenate(ops).copy(), doc_op_offsets=np.asarray(offs, dtype=np.uint64),
                  doc_init=np.asarray(init, dtype=np.uint32), clients=[[f"client-{i}" for i in range(64)]] * len(keep))
    flag_remove_order(sub.ops, sub.doc_op_offsets)
    return sub


def test_engine_remove_order_with_obliterates_matches_oracle():
    """SnapshotV1 merge info of obliterated segments (movedSeq / movedSeqs / movedClientIds,
    snapshotV1.ts:252-264) beside removedClientIds: the engine's stamps (first from rm_seq, later
    ones from the remove-order slab with their seq and kind) == the oracle's stamp lists, and the V1
    summaries are byte-identical. Parity unpinned: no reference fixture holds a V1 summary of a
    collaborative obliterate document; the oracle restates mergeTree.ts's stamp bookkeeping."""
    import oracle as orc

    batch = obliterate_v1_batch()
    eh, el, ec, ep, erm = emu_replay(batch, cap_rm=1 << 14)
    assert (eh["status"] == 0).all()
    moved = multi_moved = both = 0
    for d in range(batch.n_docs):
        want = orc.mt_removers(batch, d)
        got = summary.removers_from_engine(el[d], int(eh[d]["n_leaves"]), erm[d][: eh[d]["n_rm_order"]],
                                           _doc_ops(batch, d))
        ms = int(eh[d]["min_seq"])
        for i in range(int(eh[d]["n_leaves"])):
            rm = int(el[d][i]["rm_seq"])
            if rm != summary.NOT_REMOVED and rm > ms:
                assert got.get(i) == want.get(i), (d, i, got.get(i), want.get(i))
                kinds = [k for _, _, k in want[i]]
                moved += 1 in kinds
                multi_moved += kinds.count(1) > 1
                both += 0 in kinds and 1 in kinds
        v_en = summary.v1_summary(eh[d], el[d], ec[d], ep[d], batch.keys, batch.values, batch.clients[d], got)
        v_or = summary.v1_summary(eh[d], el[d], ec[d], ep[d], batch.keys, batch.values, batch.clients[d], want)
        assert v_en == v_or, d
    assert moved > 0 and multi_moved > 0 and both > 0, (moved, multi_moved, both)


def test_v1_moved_info_json_shape():
    """A removed-and-obliterated segment carries removedSeq/removedClient/removedClientIds, then
    movedSeq/movedSeqs/movedClientIds, in snapshotV1.ts's field order."""
    import json

    import oracle as orc

    batch = obliterate_v1_batch()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0
    seen = 0
    for d in range(batch.n_docs):
        head, bodies = summary.v1_summary(oh[d], ol[d], oc[d], op[d], batch.keys, batch.values, batch.clients[d],
                                          orc.mt_removers(batch, d))
        for blob in [head] + bodies:
            for s in json.loads(blob)["segments"]:
                if isinstance(s, dict) and "movedSeq" in s:
                    seen += 1
                    keys = list(s)
                    assert keys[-3:] == ["movedSeq", "movedSeqs", "movedClientIds"]
                    assert s["movedSeq"] == s["movedSeqs"][0] and len(s["movedSeqs"]) == len(s["movedClientIds"])
                    assert s["movedSeqs"] == sorted(s["movedSeqs"])
    assert seen > 0


def v1_reload_inputs(groups_at=(16, 40)):
    """For each reference replay fixture (tests/golden/replay_msgs_0.40.json.gz) and cut group g:
    the messages up to g are replayed by the oracle and summarized as SnapshotV1 with merge info.
    Returns [(header blob, the fixture's remaining messages, expected final text)]."""
    import gzip
    import os

    import oracle as orc

    fixtures = json.load(gzip.open(os.path.join(os.path.dirname(__file__), "golden", "replay_msgs_0.40.json.gz"),
                                   "rt", encoding="utf-8"))
    out, merge_info = [], 0
    for fx in fixtures:
        groups = fx["groups"]
        for g in groups_at:
            b1 = MergeTreeStreamBuilder()
            d = b1.begin_doc(groups[0]["initialText"], observer="A")
            for k in range(g + 1):
                for m in groups[k]["msgs"]:
                    d.add_message(m)
            batch1 = b1.finish(remove_order=True)
            rc, h, l, c, p, _ = orc.mt_replay_batch(batch1, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
            assert rc == 0
            head, bodies = summary.v1_summary(h[0], l[0], c[0], p[0], batch1.keys, batch1.values,
                                              batch1.clients[0], orc.mt_removers(batch1, 0))
            assert bodies == []
            merge_info += head.count('"json":')
            rest = [m for k in range(g + 1, len(groups)) for m in groups[k]["msgs"]]
            out.append((head, rest, groups[-1]["resultText"]))
    assert merge_info > 0
    return out


def v1_reload_batches(groups_at=(16, 40)):
    """A batch that loads each v1_reload_inputs summary (header-chunk segments with seq/client/
    removed/moved stamps) and applies the fixture's remaining messages. Returns (batch, texts)."""
    b2 = MergeTreeStreamBuilder()
    expected = []
    for head, rest, want in v1_reload_inputs(groups_at):
        d2 = b2.begin_doc_from_summary(head, [], observer="A")
        for m in rest:
            d2.add_message(m)
        expected.append(want)
    return b2.finish(), expected


def test_v1_merge_info_load_then_replay_matches_reference_text():
    """Load a SnapshotV1 summary whose segments carry merge info (specToSegment's stamps), apply the
    rest of the reference's messages: the final text is the fixture's resultText (pinned by the
    reference), and the engine (emulated) == the oracle bit for bit."""
    import oracle as orc

    batch, expected = v1_reload_batches()
    assert batch.snapshot_info is not None and len(batch.snapshot_stamps) > 0
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=512, cap_chars=2048, cap_props=1024)
    assert rc == 0
    eh, el, ec, ep = emu_replay(batch)
    for d, want in enumerate(expected):
        assert visible_text(oh[d], ol[d], oc[d]) == want, d
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_v1_body_chunk_merge_info_loads():
    """A body segment with merge info appends at the local length from its own perspective
    (snapshotLoader.ts:254-309): after a universal header it lands at the end, keeping its stamp."""
    import oracle as orc

    head = json.dumps({"version": "1", "segmentCount": 1, "length": 2, "segments": ["ab"], "startIndex": 0,
                       "headerMetadata": {"minSequenceNumber": 0, "sequenceNumber": 5, "totalLength": 3,
                                          "totalSegmentCount": 2,
                                          "orderedChunkMetadata": [{"id": "header"}, {"id": "body_0"}]}})
    body = json.dumps({"version": "1", "segmentCount": 1, "length": 1, "startIndex": 1,
                       "segments": [{"json": "c", "seq": 3, "client": "B"}]})
    b = MergeTreeStreamBuilder()
    d = b.begin_doc_from_summary(head, [body])
    d.add_message({"clientId": "B", "sequenceNumber": 6, "referenceSequenceNumber": 2, "minimumSequenceNumber": 0,
                   "type": "op", "contents": {"pos1": 2, "seg": "x", "type": 0}})
    batch = b.finish()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=512, cap_chars=2048, cap_props=1024)
    assert rc == 0 and int(oh[0]["status"]) == 0
    assert visible_text(oh[0], ol[0], oc[0]) == "abxc"  # B saw its own "c" (seq 3) at refSeq 2
    eh, el, ec, ep = emu_replay(batch)
    assert not compare_doc((oh[0], ol[0], oc[0], op[0]), (eh[0], el[0], ec[0], ep[0]))
