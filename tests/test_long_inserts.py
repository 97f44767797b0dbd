"""Inserts longer than 65535 UTF-16 units (a large paste; the reference has no limit,
mergeTree.ts:1484-1517): the op record keeps the low 16 bits in `len` and bits 16..23 in flags
(fmt.h FMT_MT_F_LEN_HI_SHIFT, fmt_mt_op_len). A 70,000-unit paste replays in the large tier, a
140,000-unit one in the huge tier; engine == oracle bit for bit, both packers byte-equal."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from fluidframework_amd.streams import MergeTreeStreamBuilder, op_len
from mt_compare import compare_doc, emu_caps, emu_huge_replay, emu_replay, visible_text

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs():
    docs = []
    for big in (70000, 140000):
        msgs = []
        seq = 0

        def m(client, ref, contents):
            nonlocal seq
            seq += 1
            msgs.append({"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                         "minimumSequenceNumber": max(0, seq - 3), "type": "op", "contents": contents})

        m("A", 0, {"pos1": 0, "seg": "hello world", "type": 0})
        m("B", 1, {"pos1": 5, "seg": "P" * big, "type": 0})  # the paste
        m("A", 1, {"pos1": 6, "seg": "xyz", "type": 0})  # concurrent, before B's paste was seen
        m("A", 3, {"pos1": 100, "pos2": 300, "type": 1})
        m("B", 4, {"pos1": big - 10, "pos2": big + 4, "props": {"bold": True}, "type": 2})
        for k in range(40):
            m("AB"[k % 2], seq, {"pos1": (k * 977) % big, "seg": "q" * (k % 5 + 1), "type": 0})
        docs.append(msgs)
    return docs


def _batch():
    b = MergeTreeStreamBuilder()
    for msgs in _docs():
        d = b.begin_doc("", observer="observer")
        for x in msgs:
            d.add_message(x)
    return b.finish()


def test_long_insert_packs_high_length_bits():
    batch = _batch()
    ins = batch.ops[batch.ops["type"] == 0]
    lens = sorted(op_len(r) for r in ins)
    assert lens[-2:] == [70000, 140000]
    assert (ins["flags"] >> 16).max() == 140000 >> 16


def test_oracle_and_emulated_tiers_on_long_inserts(orc):
    batch = _batch()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 14, cap_chars=1 << 19, cap_props=1024)
    assert rc == 0 and (oh["status"] == 0).all()
    assert int(oh[0]["visible_len"]) < 131071 < int(oh[1]["visible_len"])
    assert "P" * 1000 in visible_text(oh[1], ol[1], oc[1])
    cl, cc, cp = emu_caps(large=True)
    eh, el, ec, ep = emu_replay(batch, large=True)
    assert int(eh[0]["status"]) == 0 and int(eh[1]["status"]) == -3  # past the large tier: huge
    rc, oh0, ol0, oc0, op0, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert not compare_doc((oh0[0], ol0[0], oc0[0], op0[0]), (eh[0], el[0], ec[0], ep[0]))
    got = emu_huge_replay(batch, 1)
    assert int(got[0]["status"]) == 0
    assert compare_doc((oh[1], ol[1], oc[1], op[1]), got) == []


@pytest.mark.skipif(shutil.which("node") is None, reason="node is not installed")
def test_js_packer_long_inserts_match_python(tmp_path):
    batch = _batch()
    (tmp_path / "docs.json").write_text(json.dumps(_docs()))
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          f"const docs=JSON.parse(require('fs').readFileSync({json.dumps(str(tmp_path / 'docs.json'))},'utf8'));"
          "const b=new fmt.MergeTreeStreamBuilder();"
          "for(const msgs of docs){const d=b.beginDoc('','observer');for(const m of msgs) d.addMessage(m);}"
          "const r=b.finish();process.stdout.write(Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength).toString('hex'))")
    script = tmp_path / "long.js"
    script.write_text(js)
    r = subprocess.run(["node", str(script)], capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    assert bytes.fromhex(r.stdout) == batch.ops.tobytes()


@pytest.mark.gpu
def test_long_inserts_on_gpu(orc):
    """Through the runtime's cascade: the 70,000-unit paste finishes in the large tier, the
    140,000-unit one restarts in the huge tier — engine == oracle."""
    from fluidframework_amd import native

    batch = _batch()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 14, cap_chars=1 << 19, cap_props=1024)
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        for d in range(batch.n_docs):
            assert int(hdrs[d]["status"]) == 0, d
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)), d
    finally:
        eng.close()
