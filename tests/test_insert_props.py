"""Inserts whose segment spec carries properties: `seg: {text, props}`, what
SharedString.insertText(pos, text, props) sends (sharedString.ts:198-200). The new segment's
properties are clone(props) (TextSegment.make, textSegment.ts:41-52; BaseSegment,
mergeTreeNodes.ts:343-347): null values are dropped (properties.ts:68-95), so {"k": null} gives an
empty (defined) property set. The packers put the props-op id + 1 in the insert's pos2.

No reference fixture holds such an insert in a collaborative stream, so parity is pinned by the
oracle restatement: engine == oracle bit for bit (emulated here, the GPU in test_gpu_parity.py), the
JS packer == the Python packer byte for byte, and the catch-up op regenerated for such an insert
carries {text, props} (createInsertOp(pos, segment.clone().toJSONObject()), sequence.ts:395-452).
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from fluidframework_amd.native import PROPS_CONT

from fluidframework_amd import streams, summary
from fluidframework_amd.streams import MergeTreeStreamBuilder
from mt_compare import compare_doc, emu_caps, emu_replay

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")


def _messages():
    """Three writers with lagging refSeqs: string inserts, {text, props} inserts (one key, two keys,
    an all-null set, an empty props object), a GROUP with a props insert, annotates and removes."""
    m = []

    def add(client, seq, ref, contents, msn=0):
        m.append({"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                  "minimumSequenceNumber": msn, "contents": contents})

    add("B", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "hello ", "props": {"bold": True}}})
    add("C", 2, 0, {"type": 0, "pos1": 0, "seg": "plain "})
    add("D", 3, 1, {"type": 0, "pos1": 3, "seg": {"text": "XY", "props": {"color": "red", "bold": None}}})
    add("B", 4, 2, {"type": 0, "pos1": 5, "seg": {"text": "zz", "props": {"1": 7, "color": "blue"}}}, msn=1)
    add("C", 5, 3, {"type": 2, "pos1": 2, "pos2": 9, "props": {"bold": False}}, msn=2)
    add("D", 6, 4, {"type": 3, "ops": [{"type": 0, "pos1": 1, "seg": {"text": "g", "props": {"k": None}}},
                                       {"type": 0, "pos1": 0, "seg": {"text": "e", "props": {}}}]}, msn=3)
    add("B", 7, 5, {"type": 1, "pos1": 4, "pos2": 6}, msn=3)
    add("C", 8, 6, {"type": 0, "pos1": 2, "seg": {"text": "tail\n", "props": {"bold": True}}}, msn=3)
    add("D", 9, 8, {"type": 0, "pos1": 0, "seg": {"text": "hd", "props": {"bold": True}}}, msn=3)
    return m


def _batch(keep=False):
    b = MergeTreeStreamBuilder(keep_messages=keep)
    d = b.begin_doc("", observer="A")
    for msg in _messages():
        d.add_message(msg)
    return b.finish(catchup=keep)


def test_packer_puts_props_op_in_pos2():
    batch = _batch()
    ins = batch.ops[batch.ops["type"] == streams.MT_INSERT]
    assert [int(x) for x in ins["pos2"]] == [1, -1, 2, 3, 5, 6, 1, 1]  # (props op 3: the annotate's)
    sets = [[(batch.keys[kv >> 16], batch.values[kv & 0xFFFF]) for kv in batch.props_kv[batch.props_off[i]:batch.props_off[i + 1]]]
            for i in range(len(batch.props_off) - 1)]
    assert sets[1] == [("color", '"red"'), ("bold", "null")]
    assert sets[2] == [("1", "7"), ("color", '"blue"')]  # JS key order: array-index keys first
    assert sets[4] == [("k", "null")] and sets[5] == []


def test_oracle_and_engine_apply_insert_props(orc):
    batch = _batch()
    for large in (False, True):
        cl, cc, cp = emu_caps(large=large)
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
        assert rc == 0
        hdr, leaves, chars, props = emu_replay(batch, large=large)
        assert int(hdr[0]["status"]) == 0
        assert compare_doc((oh[0], ol[0], oc[0], op[0]), (hdr[0], leaves[0], chars[0], props[0])) == []
    # the sets the leaves hold: the two-key insert set survives as sent (JS key order), and no set
    # holds a null value (clone(props) drops them)
    h, lv, pr = oh[0], ol[0], op[0]
    used = {int(L["props"]) for L in lv[: int(h["n_leaves"])]} - {0xFFFF}
    sets = [[(batch.keys[kv >> 16], batch.values[kv & 0xFFFF]) for kv in pr[p]["kv"][: pr[p]["n"]]] for p in used]
    assert [("1", "7"), ("color", '"blue"')] in sets
    assert all(v != "null" for st in sets for _, v in st)


def test_catchup_insert_keeps_props(orc):
    batch = _batch(keep=True)
    cap = 256
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, cap_catchup=cap)
    assert rc == 0
    eh, el, ec, ep, ecu = emu_replay(batch, cap_catchup=cap)
    n = int(oh[0]["n_catchup"])
    assert int(eh[0]["n_catchup"]) == n and np.array_equal(ecu[0][:n], ocu[0][:n])
    msgs = summary.catchup_messages(batch.messages[0], ocu[0][:n], int(oh[0]["min_seq"]))
    segs = [op_["seg"] for msg in msgs for op_ in (msg["contents"]["ops"] if msg["contents"]["type"] == 3 else [msg["contents"]])
            if op_["type"] == 0]
    assert {"text": "g", "props": {}} in segs and {"text": "e", "props": {}} in segs
    assert all(isinstance(s, str) or set(s) == {"text", "props"} for s in segs)
    for s in segs:
        if isinstance(s, dict):
            assert None not in s["props"].values()


@pytest.mark.skipif(NODE is None, reason="node is not installed")
def test_js_packer_and_catchup_match_python():
    msgs = _messages()
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          f"const sm=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'summary.js'))});"
          "const b=new fmt.MergeTreeStreamBuilder();const d=b.beginDoc('','A');"
          f"for(const m of {json.dumps(msgs)}) d.addMessage(m);"
          "const r=b.finish();"
          "const ranges=[{op:0,pos1:0,pos2:0,type:0},{op:5,pos1:1,pos2:0,type:0},{op:6,pos1:0,pos2:0,type:0}];"
          f"const kept={json.dumps(msgs)}.map((m,i)=>({{message:m,firstOp:[0,1,2,3,4,5,7,8,9][i]}}));"
          "const cu=sm.catchupMessages(kept.slice(0,1).concat(kept.slice(5,6)),ranges,0);"
          "process.stdout.write(JSON.stringify({ops:Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength).toString('hex'),"
          "off:Array.from(r.propsOff),kv:Array.from(r.propsKv),cu}))")
    r = subprocess.run([NODE, "-e", js], capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py = _batch()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert out["off"] == [int(x) for x in py.props_off] and out["kv"] == [int(x) for x in py.props_kv]
    ranges = [{"op": 0, "pos1": 0, "pos2": 0, "type": 0}, {"op": 5, "pos1": 1, "pos2": 0, "type": 0},
              {"op": 6, "pos1": 0, "pos2": 0, "type": 0}]
    kept = [(m, f, 1) for m, f in zip(msgs, [0, 1, 2, 3, 4, 5, 7, 8, 9])]
    cu = summary.catchup_messages([kept[0], kept[5]], ranges, 0)
    assert json.loads(summary.catchup_blob(cu)) == out["cu"]


def _wide_messages(n_keys):
    """Writers annotating and inserting with up to n_keys keys per set, keys in differing orders,
    null deletes mixed in."""
    keys = [f"k{i}" for i in range(n_keys)]
    m = []
    seq = 0

    def add(client, ref, contents, msn=0):
        nonlocal seq
        seq += 1
        m.append({"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                  "minimumSequenceNumber": msn, "contents": contents})

    add("B", 0, {"type": 0, "pos1": 0, "seg": "abcdefghijklmnopqrstuvwxyz"})
    for r in range(12):
        ks = keys[r % 3:] + keys[: r % 3]
        props = {k: (None if (r % 4 == 3 and i == 0) else i + r) for i, k in enumerate(ks)}
        add("BCD"[r % 3], max(0, seq - 2), {"type": 2, "pos1": r % 7, "pos2": 10 + r % 9, "props": props}, msn=max(0, seq - 3))
        add("CDB"[r % 3], max(0, seq - 1), {"type": 0, "pos1": r, "seg": {"text": "+", "props": dict(reversed(list(props.items())))}},
            msn=max(0, seq - 3))
    return m


@pytest.mark.parametrize("n_keys", [5, 8, 9, 17, 40, 64, 65, 100, 128])
def test_prop_sets_up_to_128_keys_match_oracle(orc, n_keys):
    b = MergeTreeStreamBuilder()
    d = b.begin_doc("", observer="A")
    for msg in _wide_messages(n_keys):
        d.add_message(msg)
    batch = b.finish()
    assert max(int(batch.props_off[i + 1] - batch.props_off[i]) for i in range(len(batch.props_off) - 1)) == n_keys
    for large in (False, True):
        cl, cc, cp = emu_caps(large=large)
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
        assert rc == 0
        hdr, leaves, chars, props = emu_replay(batch, large=large)
        if not large and int(hdr[0]["status"]) == -3:
            continue  # more prop sets than the small tier holds: the runtime escalates to the large tier
        assert int(hdr[0]["status"]) == 0
        assert compare_doc((oh[0], ol[0], oc[0], op[0]), (hdr[0], leaves[0], chars[0], props[0])) == []
        assert max(int(p["n"]) for p in op[0][: int(oh[0]["n_props"])] if int(p["n"]) != PROPS_CONT) == n_keys


def test_prop_set_beyond_128_keys_is_a_capacity_error():
    """128 keys per set since round 6 (64 before): the working set's slots span two waves' lanes."""
    b = MergeTreeStreamBuilder()
    d = b.begin_doc("", observer="A")
    for msg in _wide_messages(129):
        d.add_message(msg)
    hdr, *_ = emu_replay(b.finish(), large=True)
    assert int(hdr[0]["status"]) == -3  # FMT_E_CAPACITY (include/fmt.h FMT_MT_PROPS_KEYS_MAX)


def _marker_messages():
    """Marker inserts (Marker.make(refType, props), mergeTreeNodes.ts:495-564) between text inserts of
    lagging writers; minSeq advances so zamboni runs: no text appends onto or across a marker."""
    m = []
    seq = 0

    def add(client, ref, contents, msn):
        nonlocal seq
        seq += 1
        m.append({"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                  "minimumSequenceNumber": msn, "contents": contents})

    add("B", 0, {"type": 0, "pos1": 0, "seg": "abcdef"}, 0)
    add("C", 1, {"type": 0, "pos1": 3, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1", "ItemType": "Paragraph"}}}, 0)
    add("D", 1, {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 0}}}, 1)
    add("B", 3, {"type": 0, "pos1": 5, "seg": "XY"}, 2)
    add("C", 3, {"type": 0, "pos1": 8, "seg": {"marker": {"refType": 0x40}, "props": {"k": None}}}, 2)
    add("D", 5, {"type": 2, "pos1": 0, "pos2": 6, "props": {"bold": True}}, 3)
    add("B", 6, {"type": 0, "pos1": 2, "seg": "zz"}, 5)
    add("C", 7, {"type": 1, "pos1": 1, "pos2": 2}, 6)
    add("D", 7, {"type": 0, "pos1": 4, "seg": "qq"}, 7)
    for k in range(20):  # text runs that zamboni merges around the markers
        add("BCD"[k % 3], seq, {"type": 0, "pos1": (k * 5) % (seq + 3), "seg": "t" + str(k)}, seq - 1)
    return m


def test_markers_match_oracle_and_keep_out_of_text(orc):
    b = MergeTreeStreamBuilder(keep_messages=True)
    d = b.begin_doc("", observer="A")
    for msg in _marker_messages():
        d.add_message(msg)
    batch = b.finish(catchup=True)
    assert int((batch.ops["flags"] & streams.MT_F_MARKER != 0).sum()) == 3
    for large in (False, True):
        cl, cc, cp = emu_caps(large=large)
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=cl, cap_chars=cc, cap_props=cp)
        assert rc == 0
        hdr, leaves, chars, props = emu_replay(batch, large=large)
        assert int(hdr[0]["status"]) == 0
        assert compare_doc((oh[0], ol[0], oc[0], op[0]), (hdr[0], leaves[0], chars[0], props[0])) == []
    lv = ol[0][: int(oh[0]["n_leaves"])]
    marks = [L for L in lv if int(L["pad"]) & streams.MT_LEAF_MARKER]
    assert len(marks) == 3 and all(int(L["len"]) == 1 for L in marks)
    assert sorted(int(oc[0][int(L["char_off"])]) for L in marks) == [0, 1, 0x40]
    # the summaries write the markers as {"marker": {"refType"}, "props"?}
    head, body = summary.legacy_summary(oh[0], ol[0], oc[0], op[0], batch.keys, batch.values)
    segs = json.loads(head)["segmentTexts"] + (json.loads(body)["segmentTexts"] if body else [])
    ms = [x for x in segs if isinstance(x, dict) and "marker" in x]
    assert len(ms) == 3 and set(ms[0]) <= {"marker", "props"}
    assert any(x["marker"] == {"refType": 1} and x["props"]["markerId"] == "m1" for x in ms)
    text = "".join(s if isinstance(s, str) else s.get("text", "") for s in segs)
    assert len(text) + 3 == json.loads(head)["totalLengthChars"]


@pytest.mark.skipif(NODE is None, reason="node is not installed")
def test_js_packer_markers_match_python():
    msgs = _marker_messages()
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          "const b=new fmt.MergeTreeStreamBuilder();const d=b.beginDoc('','A');"
          f"for(const m of {json.dumps(msgs)}) d.addMessage(m);"
          "const r=b.finish();"
          "process.stdout.write(JSON.stringify({ops:Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength).toString('hex'),"
          "text:Array.from(r.text),off:Array.from(r.propsOff),kv:Array.from(r.propsKv)}))")
    r = subprocess.run([NODE, "-e", js], capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    b = MergeTreeStreamBuilder()
    d = b.begin_doc("", observer="A")
    for msg in msgs:
        d.add_message(msg)
    py = b.finish()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert out["text"] == [int(x) for x in py.text]
    assert out["off"] == [int(x) for x in py.props_off] and out["kv"] == [int(x) for x in py.props_kv]


def test_catchup_marker_insert_json(orc):
    b = MergeTreeStreamBuilder(keep_messages=True)
    d = b.begin_doc("", observer="A")
    for msg in _marker_messages()[:6]:
        d.add_message(msg)
    batch = b.finish(catchup=True)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, cap_catchup=64)
    assert rc == 0
    n = int(oh[0]["n_catchup"])
    msgs = summary.catchup_messages(batch.messages[0], ocu[0][:n], int(oh[0]["min_seq"]))
    segs = [msg["contents"]["seg"] for msg in msgs if msg["contents"].get("type") == 0]
    assert {"marker": {"refType": 0x40}, "props": {}} in segs  # {"k": null} → properties {} (clone drops nulls)
