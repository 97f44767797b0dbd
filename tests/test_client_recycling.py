"""Short client id recycling (client.ts:831-855 getOrAddShortClientId).

Every reconnect brings a new clientId, so long-lived documents see hundreds of clients although few
write at once. The packers hand a new client the short id of a client whose stamps are all at or
below the engine's minSeq (streams.py _DocBuilder.short_client, js/fmt.js shortClient). Checks:
  * a conflict farm whose 8 writers keep reconnecting (tests/churn.py: >= 500 clientIds per
    document) packs into short ids <= 31, so it stays in the compact / small tiers;
  * the renamed stream means what the original means (it renames only at caught-up points), and the
    oracle replays both to the same state: every leaf field but the client ids, text and prop sets;
    every remove stamp above minSeq names the same writer; SnapshotV1 summaries are equal once each
    session name is mapped to its writer;
  * the engine (emulated here, the GPU in -m gpu) == the oracle on the recycled batch;
  * the JS packer packs the same bytes and the same client table.
"""
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from churn import churned_farm, session_writer
from fluidframework_amd import summary
from mt_compare import compare_doc, emu_caps, emu_replay

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def farms():
    return churned_farm(n_docs=4, ops_per_doc=3000, remove_order=True)


def _oracle(orc, batch):
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    return oh, ol, oc, op


def test_recycled_ids_fit_the_small_tier(farms):
    orig, chd, counts = farms
    assert min(counts) >= 500
    assert int(chd.ops["client"].max()) <= 31
    for d in range(chd.n_docs):
        names = chd.clients[d]
        assert len(names) <= 32 and len(set(names)) == len(names)


def test_renamed_stream_replays_to_the_same_state(orc, farms):
    orig, chd, _ = farms
    a, b = _oracle(orc, orig), _oracle(orc, chd)
    for d in range(orig.n_docs):
        ah, al, ac, ap = (x[d] for x in a)
        bh, bl, bc, bp = (x[d] for x in b)
        n = int(ah["n_leaves"])
        for f in ("n_leaves", "n_chars", "min_seq", "cur_seq", "visible_len", "n_blocks", "depth"):
            assert int(ah[f]) == int(bh[f]), (d, f)
        for f in ("ins_seq", "rm_seq", "len", "char_off", "block", "pad"):
            assert np.array_equal(al[f][:n], bl[f][:n]), (d, f)
        assert np.array_equal(ac[: int(ah["n_chars"])], bc[: int(bh["n_chars"])])
        ms = int(ah["min_seq"])
        for i in range(n):  # the writer behind each stamp above minSeq
            if int(al["ins_seq"][i]) > ms:
                assert orig.clients[d][int(al["ins_client"][i])] == session_writer(chd.clients[d][int(bl["ins_client"][i])])


def test_remove_stamps_and_v1_summaries_name_the_same_writers(orc, farms):
    orig, chd, _ = farms
    a, b = _oracle(orc, orig), _oracle(orc, chd)
    for d in range(orig.n_docs):
        ra, rb = orc.mt_removers(orig, d), orc.mt_removers(chd, d)
        ms = int(a[0][d]["min_seq"])
        n = int(a[0][d]["n_leaves"])
        for i in range(n):
            if int(a[1][d]["rm_seq"][i]) not in (summary.NOT_REMOVED,) and int(a[1][d]["rm_seq"][i]) > ms:
                wa = [(orig.clients[d][c], s, k) for c, s, k in ra[i]]
                wb = [(session_writer(chd.clients[d][c]), s, k) for c, s, k in rb[i]]
                assert wa == wb, (d, i)
        va = summary.v1_summary(a[0][d], a[1][d], a[2][d], a[3][d], orig.keys, orig.values, orig.clients[d], ra)
        vb = summary.v1_summary(b[0][d], b[1][d], b[2][d], b[3][d], chd.keys, chd.values, chd.clients[d], rb)
        strip = lambda x: re.sub(r"\b(w\d+)-\d+\b", r"\1", json.dumps(x))  # noqa: E731
        assert strip(va) == strip(vb), d
        assert re.search(r"\bw\d+-\d+\b", json.dumps(vb))  # session names above minSeq are written


def test_emulated_engine_matches_oracle_on_recycled_ids(orc, farms):
    _, chd, _ = farms
    oh, ol, oc, op = _oracle(orc, chd)
    eh, el, ec, ep, erm = emu_replay(chd, cap_rm=1 << 14)
    assert (eh["status"] == 0).all()
    for d in range(chd.n_docs):
        assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (eh[d], el[d], ec[d], ep[d])), d
        o0, o1 = int(chd.doc_op_offsets[d]), int(chd.doc_op_offsets[d + 1])
        got = summary.removers_from_engine(el[d], int(eh[d]["n_leaves"]), erm[d][: eh[d]["n_rm_order"]], chd.ops[o0:o1])
        want = orc.mt_removers(chd, d)
        assert summary.v1_summary(eh[d], el[d], ec[d], ep[d], chd.keys, chd.values, chd.clients[d], got) == \
            summary.v1_summary(oh[d], ol[d], oc[d], op[d], chd.keys, chd.values, chd.clients[d], want), d


def test_more_than_253_concurrent_writers_is_refused():
    """Recycling needs a client whose stamps are all at or below minSeq: 254 writers with stamps above
    it cannot share 253 ids (the huge tier's writer ceiling since round 6; tests/test_writer_ceiling.py)."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder, UnsupportedOp

    b = MergeTreeStreamBuilder()
    d = b.begin_doc("x", observer="o")
    with pytest.raises(UnsupportedOp):
        for k in range(254):
            d.add_message({"clientId": f"c{k}", "sequenceNumber": k + 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op",
                           "contents": {"pos1": 0, "seg": "a", "type": 0}})


@pytest.mark.skipif(shutil.which("node") is None, reason="node is not installed")
def test_js_packer_recycles_like_python(tmp_path):
    from churn import churn, farm_messages
    from fluidframework_amd import workloads

    src = workloads.conflict_farm(2, n_clients=8, ops_per_doc=2000, seed=9)
    docs = []
    for d in range(2):
        init, msgs = farm_messages(src, d)
        cm, _ = churn(msgs, seed=d)
        docs.append([init, cm])
    from churn import build

    py = build([(i, m) for i, m in docs], remove_order=True)
    script = tmp_path / "churn_pack.js"
    script.write_text(
        f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
        "const b=new fmt.MergeTreeStreamBuilder({keepMessages:true});"
        f"for(const x of JSON.parse(require('fs').readFileSync({json.dumps(str(tmp_path / 'docs.json'))},'utf8')))"
        "{const d=b.beginDoc(x[0],'observer');for(const m of x[1]) d.addMessage(m);}"
        "const r=b.finish({removeOrder:true});"
        "process.stdout.write(JSON.stringify({ops:Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength)"
        ".toString('hex'),clients:r.clients}))")
    (tmp_path / "docs.json").write_text(json.dumps(docs))
    r = subprocess.run(["node", str(script)], capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert out["clients"] == py.clients


@pytest.mark.gpu
def test_recycled_churn_farm_on_gpu(orc):
    """On the GPU: 500+ clientIds per document recycled into <= 31 short ids replay in the compact /
    small tiers only (two launches, no large-tier pass), engine == oracle bit for bit, and the V1
    summaries from GPU state name the same clients as the oracle's (plain and remove-order batches)."""
    from fluidframework_amd import native

    orig, chd, counts = churned_farm(n_docs=16, ops_per_doc=3500, seed=5, remove_order=False)
    assert min(counts) >= 500
    _, chd_rm, _ = churned_farm(n_docs=16, ops_per_doc=3500, seed=5, remove_order=True)
    eng = native.Engine(0)
    try:
        for batch, rm in ((chd, False), (chd_rm, True)):
            eng.mt_load(batch)
            eng.mt_run()
            hdrs = eng.mt_headers()
            assert (hdrs["status"] == 0).all()
            if not rm:
                assert eng.stats().launches == 2  # compact tier + small tier, no large-tier replay
            oh, ol, oc, op = _oracle(orc, batch)
            for d in range(batch.n_docs):
                lv, ch, pr = eng.mt_doc(d, hdrs[d])
                assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)), d
                if rm:
                    o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
                    got = summary.removers_from_engine(lv, int(hdrs[d]["n_leaves"]), eng.mt_remove_order(d, hdrs[d]),
                                                       batch.ops[o0:o1])
                    want = orc.mt_removers(batch, d)
                    assert summary.v1_summary(hdrs[d], lv, ch, pr, batch.keys, batch.values, batch.clients[d], got) == \
                        summary.v1_summary(oh[d], ol[d], oc[d], op[d], batch.keys, batch.values, batch.clients[d], want), d
    finally:
        eng.close()
