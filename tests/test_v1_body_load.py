"""SnapshotV1 body-chunk segments with merge info (snapshotLoader.ts:221-309).

loadBody appends each body segment through insertSegments at root.cachedLength (the local length)
from PriorPerspective(UniversalSequenceNumber, the segment's client) with its stamp, and batches
segments without merge info into one call. The hosts pack them as FMT_MT_F_LOADSEG inserts ahead of
the messages (the header alone is reloaded); the oracle and the engine apply them as the reference
does.

What the reference does with them:
- a body segment whose perspective misses an earlier segment that the local length counts (inserted
  above seq 0 by another client) cannot reach that position, and the load throws "MergeTree insert
  failed" — V1 summaries of collaborative documents with merge info in the body;
- a body whose merge-info segments come from one writer, followed by old text, loads, and replaying
  the rest of the stream reaches the original's text;
- flushBatch never clears its batch (snapshotLoader.ts:291-296): when a segment without merge info
  precedes one with merge info, every later flush inserts the batched segment objects again, aliasing
  them in the tree. The hosts refuse that shape (UnsupportedOp) instead of loading something else.
The first two are checked by oracle status and text and engine == oracle bit for bit (emulated here,
on the GPU in -m gpu), the third by both packers refusing.
"""
import json
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

from churn import farm_messages
from fluidframework_amd import summary, workloads
from fluidframework_amd.streams import MergeTreeStreamBuilder
from mt_compare import compare_doc, emu_caps, emu_huge_replay, emu_replay, visible_text


def _solo(seed, at_end, msn_lag):
    """One writer after a 12,000-unit prefix: appending at the end (at_end), or editing inside
    [11000, 11000 + its text), i.e. between the header chunk and the prefix's last 1000 units."""
    rnd, msgs, added = random.Random(seed), [], 0
    base = 12000 if at_end else 11000
    for seq in range(1, 300):
        if rnd.random() < 0.2 and added > 10:
            a = base + rnd.randint(0, added - 3)
            op = {"pos1": a, "pos2": a + 2, "type": 1}
            added -= 2
        else:
            n = rnd.randint(1, 5)
            op = {"pos1": base + (added if at_end else rnd.randint(0, added)), "seg": "q" * n, "type": 0}
            added += n
        msn = 0 if msn_lag is None else max(0, seq - msn_lag)
        msgs.append({"clientId": "solo", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                     "minimumSequenceNumber": msn, "type": "op", "contents": op})
    return "Z" * 12000, msgs


def _source_docs(msn_lag=None):
    """Collaborative farms after a 12,000-unit prefix (3), one writer appending after it (2), one
    writer editing before the prefix's tail (2). msn_lag None: the minSeq stays 0, so every segment
    inserted or removed since carries merge info; otherwise msn = seq - msn_lag."""
    src = workloads.conflict_farm(3, n_clients=8, ops_per_doc=1500, seed=3)
    docs = []
    for d in range(3):  # collaborative: the farm runs after a 12,000-unit prefix (the header chunk)
        init, msgs = farm_messages(src, d)
        for m in msgs:
            c = m["contents"]
            c["pos1"] += 12000
            if "pos2" in c:
                c["pos2"] += 12000
            if msn_lag is None:
                m["minimumSequenceNumber"] = 0
        docs.append(("Z" * 12000 + init, msgs))
    docs += [_solo(seed, True, msn_lag) for seed in (1, 2)]
    docs += [_solo(seed, False, msn_lag) for seed in (3, 4)]
    return docs


def _cut(docs, at):
    """V1 summaries of every document after its first `at` messages (oracle state), the rest of its
    messages, and the text of the whole stream."""
    import oracle as orc

    b = MergeTreeStreamBuilder(keep_messages=True)
    for init, msgs in docs:
        d = b.begin_doc(init, observer="observer")
        for m in msgs[:at]:
            d.add_message(m)
    cut = b.finish(remove_order=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(cut, cap_leaves=max(8192, 2 * at + 1024), cap_chars=1 << 17, cap_props=1024)
    assert rc == 0
    out = []
    for d, (init, msgs) in enumerate(docs):
        head, bodies = summary.v1_summary(oh[d], ol[d], oc[d], op[d], cut.keys, cut.values, cut.clients[d],
                                          orc.mt_removers(cut, d))
        assert bodies and any("json" in s for bd in bodies for s in json.loads(bd)["segments"] if isinstance(s, dict))
        out.append((head, bodies, msgs[at:]))
    return out


@pytest.fixture(scope="module")
def reload_batch():
    docs = _source_docs()
    cuts = _cut(docs, 200)
    b = MergeTreeStreamBuilder()
    for head, bodies, rest in cuts:
        d = b.begin_doc_from_summary(head, bodies)
        for m in rest:
            d.add_message(m)
    return b.finish(), docs, cuts


def test_body_with_universal_run_before_merge_info_is_refused(orc):
    """msn advancing: the older writer segments lose their merge info, so a run without merge info
    precedes segments with it and both packers refuse the body (the reference would re-insert it)."""
    from fluidframework_amd.streams import UnsupportedOp

    cuts = _cut(_source_docs(msn_lag=30)[3:5], 200)
    refused = 0
    for head, bodies, rest in cuts:
        b = MergeTreeStreamBuilder()
        segs = [s for bd in bodies for s in json.loads(bd)["segments"]]
        # a segment goes into the batch when its insert stamp is {UniversalSequenceNumber, NonCollabClient}
        stamped = [isinstance(s, dict) and "json" in s and (s.get("client") is not None or s.get("seq", 0) != 0)
                   for s in segs]
        shape_bad = any(not a and b_ for k, a in enumerate(stamped) for b_ in stamped[k + 1:])
        if shape_bad:
            with pytest.raises(UnsupportedOp):
                b.begin_doc_from_summary(head, bodies)
            refused += 1
        else:
            b.begin_doc_from_summary(head, bodies)
    assert refused == 2


def test_loader_segments_follow_the_reference(orc, reload_batch):
    batch, docs, _ = reload_batch
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    st = [int(x) for x in oh["status"]]
    # DataProcessingError "MergeTree insert failed" while loading: a farm segment whose perspective
    # misses the other writers' appended segments; the prefix's tail (a batch without merge info,
    # PriorPerspective(0, NonCollabClient)) after the writer's segments. The appending writer loads.
    assert st == [-2, -2, -2, 0, 0, -2, -2]
    assert [int(x) for x in oh["fail_seq"][5:]] == [0, 0]  # (the tail's stamp seq)
    whole = MergeTreeStreamBuilder()
    for init, msgs in docs[3:5]:
        d = whole.begin_doc(init, observer="observer")
        for m in msgs:
            d.add_message(m)
    wb = whole.finish()
    rc2, wh, wl, wc, _, _ = orc.mt_replay_batch(wb, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    for k in range(2):
        assert visible_text(oh[3 + k], ol[3 + k], oc[3 + k]) == visible_text(wh[k], wl[k], wc[k])


def test_emulated_engine_matches_oracle_on_loader_segments(orc, reload_batch):
    batch, _, _ = reload_batch
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    eh, el, ec, ep = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        assert int(eh[d]["status"]) == int(oh[d]["status"]) and int(eh[d]["fail_seq"]) == int(oh[d]["fail_seq"]), d
        if int(oh[d]["status"]) == 0:
            assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d])), d


@pytest.mark.skipif(shutil.which("node") is None, reason="node is not installed")
def test_js_packer_matches_python_on_loader_segments(reload_batch, tmp_path):
    """js/fmt.js packs the body segments as the same FMT_MT_F_LOADSEG ops as streams.py."""
    batch, _, cuts = reload_batch
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    (tmp_path / "cuts.json").write_text(json.dumps([[h, b, r] for h, b, r in cuts]))
    js = (f"const fmt=require({json.dumps(os.path.join(repo, 'fluidframework_amd', 'js', 'fmt.js'))});"
          f"const cuts=JSON.parse(require('fs').readFileSync({json.dumps(str(tmp_path / 'cuts.json'))},'utf8'));"
          "const b=new fmt.MergeTreeStreamBuilder();"
          "for(const [h,bodies,rest] of cuts){const d=b.beginDocFromSummary(h,bodies,null,'observer');"
          "for(const m of rest) d.addMessage(m);}"
          "const r=b.finish();const hex=(a)=>Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
          "process.stdout.write(JSON.stringify({ops:hex(r.ops),segs:hex(r.snapshotSegs),info:hex(r.snapshotInfo),"
          "stamps:hex(r.snapshotStamps),snaps:hex(new Uint8Array(r.snapshots))}))")
    script = tmp_path / "load.js"
    script.write_text(js)
    r = subprocess.run(["node", str(script)], capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    loader = (batch.ops["flags"] & 256) != 0
    assert loader.sum() > 100
    assert bytes.fromhex(out["ops"]) == batch.ops.tobytes()
    assert bytes.fromhex(out["segs"]) == batch.snapshot_segs.tobytes()
    assert bytes.fromhex(out["info"]) == batch.snapshot_info.tobytes()
    assert bytes.fromhex(out["stamps"]) == batch.snapshot_stamps.tobytes()
    assert bytes.fromhex(out["snaps"]) == batch.snapshots.tobytes()


@pytest.mark.gpu
def test_loader_segments_on_gpu(orc, reload_batch):
    import ctypes

    from fluidframework_amd import native

    batch, _, _ = reload_batch
    cl, cc, cp = native.capacity()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        eng.sync()
        hdrs = np.zeros(batch.n_docs, dtype=native.DOC_RESULT_DTYPE)  # fmt_mt_fetch_headers reports the failures
        native.lib().fmt_mt_fetch_headers(eng.h, hdrs.ctypes.data_as(ctypes.c_void_p))
        for d in range(batch.n_docs):
            assert int(hdrs[d]["status"]) == int(oh[d]["status"]) and int(hdrs[d]["fail_seq"]) == int(oh[d]["fail_seq"]), d
            if int(oh[d]["status"]) == 0:
                lv, ch, pr = eng.mt_doc(d, hdrs[d])
                assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)), d
    finally:
        eng.close()


def test_emulated_huge_tier_matches_oracle_on_loader_segments(orc, reload_batch):
    """The huge tier (round 5) takes loader segments as the other tiers do: insertSegments at the local
    length from PriorPerspective(UniversalSequenceNumber, client), the segment keeping its remove stamps
    (huge_engine.h loadBodySegment). Emulated with its index invariants checked after every op, normal
    and 16-slot groups: status, fail seq and state == the oracle's."""
    batch, _, _ = reload_batch
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    for tiny in (False, True):
        for d in range(batch.n_docs):
            h, lv, ch, pr = emu_huge_replay(batch, d, tiny_groups=tiny)
            assert int(h["status"]) == int(oh[d]["status"]) and int(h["fail_seq"]) == int(oh[d]["fail_seq"]), (tiny, d)
            if int(oh[d]["status"]) == 0:
                assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (h, lv, ch, pr)), (tiny, d)


def _many_segments(n, seed, rest=300):
    """One writer appends n one-unit segments after a 12,000-unit prefix (minSeq 0: none merges, every
    one keeps its merge info), then edits inside them: the V1 summary after the appends has a body of
    about n segments with merge info, the messages after it continue the stream."""
    rnd, msgs = random.Random(seed), []
    for k in range(n):
        msgs.append({"clientId": "solo", "sequenceNumber": k + 1, "referenceSequenceNumber": k,
                     "minimumSequenceNumber": 0, "type": "op", "contents": {"pos1": 12000 + k, "seg": "abcdefgh"[k % 8], "type": 0}})
    length = 12000 + n
    for j in range(rest):
        seq = n + j + 1
        if rnd.random() < 0.3:
            a = rnd.randint(12000, length - 3)
            op = {"pos1": a, "pos2": a + 2, "type": 1}
            length -= 2
        else:
            op = {"pos1": rnd.randint(12000, length), "seg": "x" * rnd.randint(1, 4), "type": 0}
            length += len(op["seg"])
        msgs.append({"clientId": "solo", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                     "minimumSequenceNumber": 0, "type": "op", "contents": op})
    return "Z" * 12000, msgs


def _many_segments_batch(n, seed=31):
    init, msgs = _many_segments(n, seed)
    (head, bodies, rest), = _cut([(init, msgs)], n)
    b = MergeTreeStreamBuilder()
    d = b.begin_doc_from_summary(head, bodies)
    for m in rest:
        d.add_message(m)
    batch = b.finish()
    assert ((batch.ops["flags"] & 256) != 0).sum() > n // 2
    return batch, init, msgs


def test_emulated_huge_tier_loads_a_long_v1_body(orc):
    """A V1 body of 2,500 segments with merge info, loaded and edited in the huge tier (emulated) ==
    the oracle, whose text equals the unsummarized stream's."""
    batch, init, msgs = _many_segments_batch(2500)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=16384, cap_chars=1 << 17, cap_props=1024)
    assert rc == 0
    h, lv, ch, pr = emu_huge_replay(batch, 0)
    assert not compare_doc((oh[0], ol[0], oc[0], op[0]), (h, lv, ch, pr))
    whole = MergeTreeStreamBuilder()
    d = whole.begin_doc(init, observer="observer")
    for m in msgs:
        d.add_message(m)
    rc2, wh, wl, wc, _, _ = orc.mt_replay_batch(whole.finish(), cap_leaves=16384, cap_chars=1 << 17, cap_props=1024)
    assert visible_text(oh[0], ol[0], oc[0]) == visible_text(wh[0], wl[0], wc[0])


@pytest.mark.gpu
def test_long_v1_body_loads_in_the_huge_tier_on_gpu(orc):
    """A V1 summary whose body holds 20,000 segments with merge info: past the large tier at load, so
    the runtime routes it to the huge tier, whose loader segments replay it == the oracle."""
    from fluidframework_amd import native

    batch, _, _ = _many_segments_batch(20000)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=65536, cap_chars=1 << 18, cap_props=1024)
    assert rc == 0
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        lv, ch, pr = eng.mt_doc(0, hdrs[0])
        assert not compare_doc((oh[0], ol[0], oc[0], op[0]), (hdrs[0], lv, ch, pr))
        assert eng.huge_profile(0)["replay"] > 0  # (it ran in the huge tier)
    finally:
        eng.close()
