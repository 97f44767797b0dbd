"""The N-API addon (fluidframework_amd/fmt_napi.node) and the JavaScript batch driver (js/fmt.js).

CPU: the addon loads in the image's Node and exports its functions; opening a context without a GPU
rejects with FMT_E_DEVICE; the JavaScript packer produces byte-identical records to streams.py for
the reference's replay fixtures (tests/golden/replay_msgs_0.40.json.gz, the messages
client.replay.spec.ts:20-76 replays).
GPU: every checkpoint of those fixtures replayed from JavaScript through the addon matches the
fixture's resultText; summarize() from GPU state (legacy blobs + catch-up ops) equals the Python
host's; a SharedMap bunch replay gives the LWW entries in JS Map order and its summary.
"""
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "fluidframework_amd")
ADDON = os.path.join(PKG, "fmt_napi.node")
DRIVER = os.path.join(REPO, "tests", "js", "fixture_driver.js")
GOLDEN = os.path.join(REPO, "tests", "golden", "replay_msgs_0.40.json.gz")

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


@pytest.fixture(scope="module")
def addon():
    if not os.path.exists(ADDON):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "napi")], check=True)
    return ADDON


def _node(*args, timeout=120):
    # (FMT_NAPI_BACKTRACE: a SIGSEGV in the child prints its native stack into r.stderr, which the
    # assertions show — INTEGRATION.md §2, the open exit-path crash)
    env = dict(os.environ, FMT_NAPI_BACKTRACE=os.environ.get("FMT_NAPI_BACKTRACE", "1"))
    return subprocess.run([NODE, *args], capture_output=True, text=True, timeout=timeout, cwd=REPO, env=env)


def test_addon_exports(addon):
    r = _node("-e", f"const a=require({json.dumps(addon)});"
                    "console.log(JSON.stringify({k:Object.keys(a).sort(),s:a.sizes,c:a.capacity()}))")
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["k"] == sorted(["open", "close", "openContexts", "deviceInfo", "capacity", "stats", "replayMergeTree", "fetchCatchup",
                               "fetchRemoveOrder", "fetchNumbers", "fetchLegacyProps", "fetchRmClientsHi", "fetchRegen", "replayMapSparse", "summarizeLegacy", "fetchCatchupAll",
                               "summaryBlobs", "replayMap", "fetchDoc", "sizes"])
    assert out["s"] == {"mtOp": 32, "mapOp": 16, "leaf": 32, "docResult": 48, "propset": 36, "mapSlot": 8,
                        "catchupRange": 16, "mapEntry": 12, "adjust": 32}
    assert out["c"]["leaves"] >= 512


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_open_without_gpu_rejects(addon):
    r = _node("-e", "const f=require('./fluidframework_amd/js/fmt.js');"
                    "try{new f.Engine(0);console.log('opened')}catch(e){console.log(e.code)}")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "FMT_E_DEVICE"


@pytest.mark.gpu
def test_contexts_open_close_churn_and_cap(addon):
    """Context lifetime (fmt_napi.cc, no N-API finalizers): 200 open/close cycles leave no context
    open (the slot table is reused); contexts dropped without close() count against the cap
    (FMT_NAPI_MAX_CONTEXTS) so device memory cannot grow without bound, close() of a stale handle is
    a no-op and using it throws; the env cleanup hook closes what is still open and node exits 0."""
    js = (f"const a=require({json.dumps(addon)});"
          "for(let i=0;i<200;i++){const c=a.open(0);a.close(c);}"
          "const n0=a.openContexts();"
          "let capped='';const held=[];"
          "try{for(let i=0;i<8;i++) held.push(a.open(0));}catch(e){capped=e.code;}"
          "const n1=a.openContexts();"
          "a.close(held[0]);a.close(held[0]);let stale='';"
          "try{a.deviceInfo(held[0]);}catch(e){stale=e.code;}"
          "process.stdout.write(JSON.stringify({n0,n1,capped,stale,n2:a.openContexts()}));")
    env = dict(os.environ, FMT_NAPI_MAX_CONTEXTS="5")
    r = subprocess.run([NODE, "-e", js], capture_output=True, text=True, timeout=120, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out == {"n0": 0, "n1": 5, "capped": "FMT_E_CAPACITY", "stale": "FMT_E_USAGE", "n2": 4}


def _python_pack(stride):
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    fixtures = json.load(gzip.open(GOLDEN, "rt", encoding="utf-8"))
    b = MergeTreeStreamBuilder()
    for fx in fixtures:
        groups = fx["groups"]
        for k in range(0, len(groups), stride):
            d = b.begin_doc(initial_text=groups[0]["initialText"], observer="A")
            for g in range(k + 1):
                for m in groups[g]["msgs"]:
                    d.add_message(m)
    return b.finish()


def test_js_packer_matches_python_packer(addon, tmp_path):
    r = _node(DRIVER, "pack", str(tmp_path))
    assert r.returncode == 0, r.stderr
    py = _python_pack(8)
    rd = lambda n, dt: np.fromfile(tmp_path / n, dtype=dt)  # noqa: E731
    assert rd("ops.bin", np.uint8).tobytes() == py.ops.tobytes()
    assert np.array_equal(rd("offs.bin", np.uint64), py.doc_op_offsets)
    assert np.array_equal(rd("text.bin", "<u2"), py.text)
    assert np.array_equal(rd("doc_init.bin", np.uint32), py.doc_init.reshape(-1))
    assert np.array_equal(rd("props_off.bin", np.uint32), py.props_off)
    assert np.array_equal(rd("props_kv.bin", np.uint32), py.props_kv)
    meta = json.load(open(tmp_path / "meta.json"))
    assert meta["keys"] == py.keys and meta["values"] == py.values and meta["clients"] == py.clients


def test_js_packer_sided_obliterate_matches_python(addon):
    """Type 5 places {pos, before} pack as pos + FMT_MT_F_START_BEFORE / FMT_MT_F_END_BEFORE, alone
    and as a GROUP member (with FMT_MT_F_GROUP_CONT), identically in the JS and Python packers."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    sided = {"type": 5, "pos1": {"pos": 1, "before": False}, "pos2": {"pos": 3, "before": True}}
    msgs = [
        {"clientId": "B", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
         "contents": sided},
        {"clientId": "C", "sequenceNumber": 2, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
         "contents": {"type": 3, "ops": [{"type": 1, "pos1": 0, "pos2": 1},
                                          {"type": 5, "pos1": {"pos": 0, "before": True},
                                           "pos2": {"pos": 1, "before": False}}]}},
    ]
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          "const b=new fmt.MergeTreeStreamBuilder();const d=b.beginDoc('abcdef','A');"
          f"for(const m of {json.dumps(msgs)}) d.addMessage(m);"
          "const r=b.finish();process.stdout.write(Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength).toString('hex'))")
    r = _node("-e", js)
    assert r.returncode == 0, r.stderr
    sb = MergeTreeStreamBuilder()
    d = sb.begin_doc("abcdef")
    for m in msgs:
        d.add_message(m)
    py = sb.finish()
    assert bytes.fromhex(r.stdout.strip()) == py.ops.tobytes()
    assert [int(f) for f in py.ops["flags"]] == [16, 0, 8 | 1]


def test_js_packer_refuses_ambiguous_marker_ids(addon):
    """Mirror of test_relative_pos.py::test_ambiguous_marker_ids_are_refused in the JS packer."""
    msgs = [
        {"clientId": "B", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
         "contents": {"type": 0, "pos1": 1, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m"}}}},
        {"clientId": "B", "sequenceNumber": 2, "referenceSequenceNumber": 1, "minimumSequenceNumber": 0,
         "contents": {"type": 2, "pos1": 1, "pos2": 2, "props": {"markerId": "n"}}},
        {"clientId": "C", "sequenceNumber": 3, "referenceSequenceNumber": 2, "minimumSequenceNumber": 0,
         "contents": {"type": 0, "relativePos1": {"id": "n"}, "seg": "X"}},
    ]
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          "const b=new fmt.MergeTreeStreamBuilder();const d=b.beginDoc('abc','A');"
          f"const m={json.dumps(msgs)};d.addMessage(m[0]);d.addMessage(m[1]);"
          "try{d.addMessage(m[2]);console.log('packed')}catch(e){console.log(e.name+':'+(e instanceof fmt.UnsupportedOp))}")
    r = _node("-e", js)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith(":true"), r.stdout


def test_js_map_packer_orders_bunches(addon):
    """Messages of one bunch share a sequenceNumber; the packer keeps their order via the ordinal."""
    r = _node("-e", """
const f=require('./fluidframework_amd/js/fmt.js');
const b=new f.MapStreamBuilder(); const d=b.beginDoc();
b.processMessagesCore(d,{envelope:{sequenceNumber:5},local:false,messagesContent:[
 {contents:{type:'delete',key:'k'}},{contents:{type:'set',key:'k',value:{type:'Plain',value:1}}}]});
const x=b.finish(); const v=new DataView(x.ops.buffer);
console.log(JSON.stringify([v.getUint32(8,true),v.getUint32(24,true),x.keyBound,x.values]));""")
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout) == [1, 2, 1, ["1"]]


def test_js_summary_load_packing_matches_python(addon, orc, tmp_path):
    """beginDocFromSummary packs legacy summaries (with catch-up blobs) exactly like streams.py."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder
    from test_snapshot_load import summaries_of
    from test_catchup import fixture_batch

    batch, _ = fixture_batch()
    sums = [s[:3] for s in summaries_of(orc, batch)]
    (tmp_path / "in.json").write_text(json.dumps(sums))
    r = _node(DRIVER, "packsummaries", str(tmp_path / "in.json"), str(tmp_path / "out"))
    assert r.returncode == 0, r.stderr
    b = MergeTreeStreamBuilder()
    for h, body, cu in sums:
        b.begin_doc_from_summary(h, body, cu)
    py = b.finish()
    out = tmp_path / "out"
    assert (out / "ops.bin").read_bytes() == py.ops.tobytes()
    assert (out / "text.bin").read_bytes() == py.text.tobytes()
    assert (out / "snapshots.bin").read_bytes() == py.snapshots.tobytes()
    assert (out / "snapshot_segs.bin").read_bytes() == py.snapshot_segs.tobytes()
    assert (out / "props_kv.bin").read_bytes() == py.props_kv.tobytes()


@pytest.mark.gpu
def test_js_replay_all_fixture_checkpoints_on_gpu(addon):
    r = _node(DRIVER, "replay", timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["checked"] == 6 * 64
    assert out["nMismatches"] == 0, out["mismatches"]
    assert "gfx950" in out["device"]


@pytest.mark.gpu
def test_js_map_bunches_on_gpu(addon):
    r = _node(DRIVER, "map", timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # doc0: b,a set; delete b then set b (moves to the end); a updated in place (mapKernel.ts:708-850)
    assert out["doc0"] == [["a", "y"], ["b", {"n": [1, 2]}]]
    assert out["doc1"] == [["c", True]]
    assert out["a0"] == "y"
    assert out["summary0"] == ('{"blobs":[],"content":{"a":{"type":"Plain","value":"y"},'
                               '"b":{"type":"Plain","value":{"n":[1,2]}}}}')


@pytest.mark.gpu
def test_js_legacy_summaries_with_catchup_on_gpu(addon, orc):
    """summarize() from GPU state through the addon == the Python host over the oracle's state."""
    from fluidframework_amd import summary
    from test_catchup import CAP, fixture_batch

    r = _node(DRIVER, "summary", timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    batch, _ = fixture_batch()
    rc, h, leaves, chars, props, _, cu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    assert rc == 0 and len(got) == batch.n_docs
    for d in range(batch.n_docs):
        head, body = summary.legacy_summary(h[d], leaves[d], chars[d], props[d], batch.keys, batch.values)
        msgs = summary.catchup_messages(batch.messages[d], cu[d][: h[d]["n_catchup"]], int(h[d]["min_seq"]))
        assert got[d]["header"] == head and got[d]["body"] == body, d
        assert got[d]["catchupOps"] == summary.catchup_blob(msgs), d


@pytest.mark.gpu
def test_js_v1_summaries_on_gpu(addon, orc):
    """summarizeV1() from GPU state (remove-order slab through the addon) == the Python host over
    the oracle's state and remove stamps."""
    from fluidframework_amd import summary
    from test_snapshot_v1 import _collab_batch

    r = _node(DRIVER, "v1", timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    batch = _collab_batch()
    rc, h, leaves, chars, props, _ = orc.mt_replay_batch(batch, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0 and len(got) == batch.n_docs
    for d in range(batch.n_docs):
        head, bodies = summary.v1_summary(h[d], leaves[d], chars[d], props[d], batch.keys, batch.values,
                                          batch.clients[d], orc.mt_removers(batch, d))
        assert got[d]["header"] == head and got[d]["bodies"] == bodies, d


def _relative_messages():
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_relative_pos import hand_cases

    return hand_cases()


def test_js_packer_relative_positions_match_python(addon):
    """relativePos1/2 pack as FMT_MT_F_REL1/REL2 ops indexing the relpos table, with the marker id
    interned as the value its "markerId" property holds, identically in the JS and Python packers."""
    from test_relative_pos import _batch

    cases = _relative_messages()
    docs = [{"init": init, "msgs": msgs} for msgs, init, _ in cases]
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          "const b=new fmt.MergeTreeStreamBuilder();"
          f"for(const x of {json.dumps(docs)}){{const d=b.beginDoc(x.init,'A');for(const m of x.msgs) d.addMessage(m);}}"
          "const r=b.finish();const hex=(a)=>Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
          "process.stdout.write(JSON.stringify({ops:hex(r.ops),relpos:hex(r.relpos),key:r.markerIdKey,"
          "keys:r.keys,values:r.values}))")
    r = _node("-e", js)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py = _batch(cases)
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert bytes.fromhex(out["relpos"]) == py.relpos.tobytes()
    assert out["key"] == py.marker_id_key and out["keys"] == py.keys and out["values"] == py.values


@pytest.mark.gpu
def test_js_relative_positions_on_gpu(addon):
    """The JS driver replays relativePos ops through the addon; getText equals the hand cases."""
    cases = _relative_messages()
    docs = [{"init": init, "msgs": msgs} for msgs, init, _ in cases]
    js = (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
          "(async()=>{const b=new fmt.MergeTreeStreamBuilder();"
          f"for(const x of {json.dumps(docs)}){{const d=b.beginDoc(x.init,'A');for(const m of x.msgs) d.addMessage(m);}}"
          "const e=new fmt.Engine(0);const r=await e.replayMergeTree(b.finish());"
          f"const t=[];for(let i=0;i<{len(cases)};i++) t.push(r.getText(i));e.close();"
          "process.stdout.write(JSON.stringify(t));})().catch((e)=>{console.error(e);process.exit(1);});")
    r = _node("-e", js, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout) == [want for _, _, want in cases]


def _v1_reload_js(cases):
    docs = [{"head": h, "msgs": m} for h, m, _ in cases]
    return (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
            "const b=new fmt.MergeTreeStreamBuilder();"
            f"for(const x of {json.dumps(docs)}){{const d=b.beginDocFromSummary(x.head,[],null,'A');"
            "for(const m of x.msgs) d.addMessage(m);}")


def test_js_v1_merge_info_load_matches_python(addon, tmp_path):
    """SnapshotV1 header chunks with merge info load through the JS packer into the same segment
    specs, merge-info rows and stamps as the Python host's (begin_doc_from_summary)."""
    from test_snapshot_v1 import v1_reload_batches, v1_reload_inputs

    cases = v1_reload_inputs()
    js = _v1_reload_js(cases) + (
        "const r=b.finish();const hex=(a)=>a===undefined?'':Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
        "process.stdout.write(JSON.stringify({ops:hex(r.ops),segs:hex(r.snapshotSegs),info:hex(r.snapshotInfo),"
        "stamps:hex(r.snapshotStamps),snaps:hex(new Uint8Array(r.snapshots)),clients:r.clients}))")
    script = tmp_path / "v1_load.js"
    script.write_text(js)
    r = _node(str(script), timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py, _ = v1_reload_batches()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert bytes.fromhex(out["segs"]) == py.snapshot_segs.tobytes()
    assert bytes.fromhex(out["info"]) == py.snapshot_info.tobytes()
    assert bytes.fromhex(out["stamps"]) == py.snapshot_stamps.tobytes()
    assert bytes.fromhex(out["snaps"]) == py.snapshots.tobytes()
    assert out["clients"] == py.clients


@pytest.mark.gpu
def test_js_v1_merge_info_load_on_gpu(addon, tmp_path):
    """The JS driver loads mid-stream V1 summaries with merge info, replays the rest of the
    reference's messages through the addon, and reaches the fixtures' resultText."""
    from test_snapshot_v1 import v1_reload_inputs

    cases = v1_reload_inputs()
    js = ("(async()=>{" + _v1_reload_js(cases) + "const e=new fmt.Engine(0);const r=await e.replayMergeTree(b.finish());"
          f"const t=[];for(let i=0;i<{len(cases)};i++) t.push(r.getText(i));e.close();"
          "process.stdout.write(JSON.stringify(t));})().catch((e)=>{console.error(e);process.exit(1);});")
    script = tmp_path / "v1_load_gpu.js"
    script.write_text(js)
    r = _node(str(script), timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout) == [want for _, _, want in cases]


def _adjust_js(docs, body):
    return (f"const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});"
            "const b=new fmt.MergeTreeStreamBuilder();"
            f"for(const x of {json.dumps(docs)}){{const d=b.beginDoc(x[0],'A');for(const m of x[1]) d.addMessage(m);}}" + body)


def test_js_packer_annotate_adjust_matches_python(addon, tmp_path):
    """Annotate-adjust packs identically in the JS and Python packers: the props ops with their
    (key, FMT_MT_VALUE_ADJUST) + row entries, the fmt_mt_adjust rows, and each value's number."""
    from test_annotate_adjust import adjust_fixture_batch

    docs = adjust_fixture_batch(messages=True)
    script = tmp_path / "adj_pack.js"
    script.write_text(_adjust_js(docs, (
        "const r=b.finish();const hex=(a)=>Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
        "process.stdout.write(JSON.stringify({ops:hex(r.ops),off:hex(r.propsOff),kv:hex(r.propsKv),adj:hex(r.adjusts),"
        "num:hex(r.valueNum),values:r.values}))")))
    r = _node(str(script))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py, _ = adjust_fixture_batch()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert bytes.fromhex(out["off"]) == py.props_off.tobytes() and bytes.fromhex(out["kv"]) == py.props_kv.tobytes()
    assert bytes.fromhex(out["adj"]) == py.adjusts.tobytes()
    assert bytes.fromhex(out["num"]) == py.value_num.tobytes()
    assert out["values"] == py.values


@pytest.mark.gpu
def test_js_annotate_adjust_summaries_on_gpu(addon, tmp_path, orc):
    """Through the addon: getText equals the fixtures' resultText; summarizeV1 (computed numbers as
    JSON.stringify writes them) equals the Python host over the GPU state; every legacy summary
    (getAtSeq(minSeq) from fetchLegacyProps) equals the oracle's SnapshotLegacy restatement."""
    from fluidframework_amd import native
    from fluidframework_amd.summary import v1_summary, values_with_numbers, removers_from_engine
    from test_annotate_adjust import adjust_fixture_batch

    for exact_tail in (True, False):
        docs = adjust_fixture_batch(exact_tail=exact_tail, messages=True)
        script = tmp_path / f"adj_gpu_{exact_tail}.js"
        script.write_text("(async()=>{" + _adjust_js(docs, (
            "const e=new fmt.Engine(0);const r=await e.replayMergeTree(b.finish());const out=[];"
            f"for(let i=0;i<{len(docs)};i++){{let leg=null;try{{leg=r.summarize(i)}}catch(x){{leg=x.code}}"
            "out.push({text:r.getText(i),v1:r.summarizeV1(i),legacy:leg});}"
            "e.close();process.stdout.write(JSON.stringify(out));})().catch((e)=>{console.error(e);process.exit(1);});")))
        r = _node(str(script), timeout=300)
        assert r.returncode == 0, r.stderr
        out = json.loads(r.stdout)
        batch, finals = adjust_fixture_batch(exact_tail)
        for d, o in enumerate(out):
            assert o["text"] == finals[d]
            assert not isinstance(o["legacy"], str), (d, o["legacy"])
            want = orc.mt_replay_summary(batch, d, batch.keys, batch.values)
            assert [o["legacy"]["header"], o["legacy"].get("body")] == list(want), d
        e = native.Engine(0)
        try:
            e.mt_load(batch)
            e.mt_run()
            hdrs = e.mt_headers()
            for d, o in enumerate(out):
                lv, ch, pr = e.mt_doc(d, hdrs[d])
                vals = values_with_numbers(batch.values, e.mt_numbers(d))
                a, bb = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
                rem = removers_from_engine(lv, int(hdrs[d]["n_leaves"]), e.mt_remove_order(d, hdrs[d]), batch.ops[a:bb])
                head, bodies = v1_summary(hdrs[d], lv, ch, pr, batch.keys, vals, batch.clients[d], rem)
                assert [o["v1"]["header"], o["v1"]["bodies"]] == [head, bodies], d
        finally:
            e.close()


@pytest.mark.gpu
def test_js_sparse_map_and_bulk_summaries_on_gpu(addon, tmp_path):
    """The addon's sparse map path (replayMapSparse, key pools of any size) gives the dense path's live
    entries and summaries; the bulk legacy summaries (summarizeAllLegacy: device merge + C++ JSON)
    equal the JS host's per-document summarize() on the reference's replay fixtures."""
    js = f"""const fmt=require({json.dumps(os.path.join(REPO, 'fluidframework_amd', 'js', 'fmt.js'))});
const zlib=require('zlib');const fs=require('fs');
(async()=>{{
const mb=new fmt.MapStreamBuilder();let x=12345;const rnd=(n)=>{{x=(x*1103515245+12345)%2147483648;return x%n;}};
for(let d=0;d<64;d++){{const doc=mb.beginDoc();for(let s=1;s<=600;s++){{const r=rnd(41);
 const c=r<20?{{type:'set',key:'k'+rnd(3000),value:{{type:'Plain',value:rnd(50)}}}}:(r<40?{{type:'delete',key:'k'+rnd(3000)}}:{{type:'clear'}});
 mb.addMessage(doc,s,c);}}}}
const mbatch=mb.finish();const e=new fmt.Engine(0);
const dense=await e.replayMap(mbatch);const sparse=await e.replayMapSparse(mbatch);
const out={{map:[]}};
for(let d=0;d<64;d++) out.map.push([JSON.stringify(dense.entries(d))===JSON.stringify(sparse.entries(d)),
  JSON.stringify(dense.summarize(d))===JSON.stringify(sparse.summarize(d)), sparse.entries(d).length]);
const fx=JSON.parse(zlib.gunzipSync(fs.readFileSync({json.dumps(GOLDEN)})).toString());
const b=new fmt.MergeTreeStreamBuilder({{keepMessages:true}});
for(const f of fx){{const d=b.beginDoc(f.groups[0].initialText,'A');for(const g of f.groups) for(const m of g.msgs) d.addMessage(m);}}
const r=await e.replayMergeTree(b.finish({{catchup:true}}));const t=await r.summarizeAllLegacy();out.bytes=t.bytes;out.legacy=[];out.cu=0;
for(let d=0;d<fx.length;d++){{const a=r.legacyBlobs(d),h=r.summarize(d);out.cu+=a.catchupOps!==undefined;
 out.legacy.push(a.header===h.header&&a.body===h.body&&a.catchupOps===h.catchupOps);}}
e.close();process.stdout.write(JSON.stringify(out));}})().catch((e)=>{{console.error(e);process.exit(1);}});"""
    script = tmp_path / "sparse_bulk.js"
    script.write_text(js)
    r = _node(str(script), timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert all(a and b for a, b, _ in out["map"]) and sum(n for _, _, n in out["map"]) > 1000
    assert out["bytes"] > 0 and all(out["legacy"]) and out["cu"] > 0  # catchupOps from the bulk copy too


def test_js_packer_document_local_values_match_python(addon, tmp_path):
    """A batch with more distinct property values than 16-bit batch-global ids (each Marker's own
    markerId): the JS packer switches to document-local ids (docValueBase, fmt.h doc_value_base)
    exactly as streams.py does — the same op records, props tables, values and bases."""
    import marker_docs

    docs = [marker_docs.doc_messages(d, 1200, 3) for d in range(200)]
    (tmp_path / "docs.json").write_text(json.dumps([{"init": i, "msgs": m} for i, m in docs]))
    script = (
        "const f=require('./fluidframework_amd/js/fmt.js');const fs=require('fs');"
        f"const out={json.dumps(str(tmp_path))};"
        "const docs=JSON.parse(fs.readFileSync(out+'/docs.json','utf8'));"
        "const b=new f.MergeTreeStreamBuilder();"
        "for(const x of docs){const d=b.beginDoc(x.init);for(const m of x.msgs)d.addMessage(m);}"
        "const r=b.finish();"
        "fs.writeFileSync(out+'/ops.bin',Buffer.from(r.ops.buffer,r.ops.byteOffset,r.ops.byteLength));"
        "fs.writeFileSync(out+'/props_off.bin',Buffer.from(r.propsOff.buffer));"
        "fs.writeFileSync(out+'/props_kv.bin',Buffer.from(r.propsKv.buffer));"
        "fs.writeFileSync(out+'/relpos.bin',Buffer.from(r.relpos.buffer));"
        "fs.writeFileSync(out+'/base.bin',Buffer.from(r.docValueBase.buffer));"
        "fs.writeFileSync(out+'/meta.json',JSON.stringify({values:r.values}));")
    r = _node("-e", script, timeout=600)
    assert r.returncode == 0, r.stderr
    py = marker_docs.marker_batch(200, 1200, seed=3)
    assert py.value_base is not None
    rd = lambda n, dt: np.fromfile(tmp_path / n, dtype=dt)  # noqa: E731
    assert rd("ops.bin", np.uint8).tobytes() == py.ops.tobytes()
    assert np.array_equal(rd("props_off.bin", np.uint32), py.props_off)
    assert np.array_equal(rd("props_kv.bin", np.uint32), py.props_kv)
    assert rd("relpos.bin", np.uint8).tobytes() == py.relpos.tobytes()
    assert np.array_equal(rd("base.bin", np.uint32), py.value_base)
    assert json.load(open(tmp_path / "meta.json"))["values"] == py.values


def _pending_js(body):
    """A JS program that rebuilds the map pending scenarios (tests/golden/map_pending_cases.json) with
    fmt.js's MapStreamBuilder, one document per assertion as test_map_pending.golden_checkpoints does."""
    gold = os.path.join(REPO, "tests", "golden", "map_pending_cases.json")
    return (f"const fmt=require({json.dumps(os.path.join(PKG, 'js', 'fmt.js'))});"
            f"const cases=JSON.parse(require('fs').readFileSync({json.dumps(gold)},'utf8')).cases;"
            "const plain=(o)=>o.type!=='set'?o:{type:'set',key:o.key,value:{type:'Plain',value:o.value}};"
            "const b=new fmt.MapStreamBuilder();const checks=[];"
            "for(const c of cases){c.steps.forEach((st,si)=>{if(!st[0].startsWith('expect'))return;"
            "const d=b.beginDoc();let seq=0;for(const s of c.steps.slice(0,si)){"
            "if(s[0]==='local')b.localSubmit(d,plain(s[1]));"
            "else if(s[0]==='flush'){while(b.unacked.length)b.localAck(d,++seq);}"
            "else if(s[0]==='remote')b.addMessage(d,++seq,plain(s[1]));"
            "else if(s[0]==='rollback_all'){while(b.unacked.length)b.localRollback(d);}}"
            "checks.push([d,st]);});}const batch=b.finish();" + body)


def test_js_map_pending_packing_matches_python(addon, tmp_path):
    """fmt.js packs the local client's events (localSubmit / localAck / localRollback) into the same
    fmt_map_local_op records and sequenced ops as the Python host."""
    from test_map_pending import golden_checkpoints

    script = tmp_path / "pending_pack.js"
    script.write_text(_pending_js(
        "const hex=(a)=>Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
        "process.stdout.write(JSON.stringify({ops:hex(batch.ops),ev:hex(batch.localOps),"
        "eo:Array.from(batch.localOffsets,Number),keys:batch.keys,values:batch.values}));"))
    r = _node(str(script))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py = golden_checkpoints()[0].finish()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert bytes.fromhex(out["ev"]) == py.local_ops.tobytes()
    assert out["eo"] == py.local_offsets.tolist()
    assert out["keys"] == py.keys and out["values"] == py.values


@pytest.mark.gpu
def test_js_map_pending_view_on_gpu(addon, tmp_path):
    """The JS driver's optimistic view (replayMapSparse with localOps, SparseMapReplay
    .optimisticEntries) reaches what the reference's rollback / iteration tests assert."""
    from test_map_pending import _check_assertion, golden_checkpoints

    script = tmp_path / "pending_gpu.js"
    script.write_text("(async()=>{" + _pending_js(
        "const e=new fmt.Engine(0);const r=await e.replayMapSparse(batch);"
        "const out=checks.map(([d,st])=>[r.optimisticEntries(d),st]);e.close();"
        "process.stdout.write(JSON.stringify(out));") + "})().catch((e)=>{console.error(e);process.exit(1);});")
    r = _node(str(script), timeout=300)
    assert r.returncode == 0, r.stderr
    checks = json.loads(r.stdout)
    assert len(checks) == len(golden_checkpoints()[1])
    for view, step in checks:
        _check_assertion([tuple(x) for x in view], step)


# ---- f4: the merge-tree local client (submissions, acks, rollbacks, reconnects) from JavaScript --

_LOCAL_JS = (
    "const fs=require('fs');const fmt=require(%s);const log=JSON.parse(fs.readFileSync(%s,'utf8'));"
    "const b=new fmt.MergeTreeStreamBuilder();const docs={};"
    "for(const e of log){const d=docs[e[0]];"
    "if(e[1]==='begin')docs[e[0]]=b.beginDoc(e[2],e[3]);"
    "else if(e[1]==='local_op')d.localOp(e[2]);else if(e[1]==='add_message')d.addMessage(e[2]);"
    "else if(e[1]==='local_rollback')d.localRollback();else if(e[1]==='local_regen')d.localRegen(e[2]||undefined,e[3]);"
    "else if(e[1]==='regen_pending')d.regenPending(e[2]);else throw new Error(e[1]);}"
    "const batch=b.finish();")


def _local_log(tmp_path, seeds=(3, 4), steps=300, **kw):
    from local_farm import farm_log, local_farm_batch

    _, farms = local_farm_batch(seeds, steps=steps, **kw)
    log = farm_log(farms)
    path = tmp_path / "local_log.json"
    path.write_text(json.dumps(log))
    return log, path


@pytest.mark.parametrize("new_ids", [False, True])
def test_js_packer_local_client_matches_python(addon, tmp_path, new_ids):
    """fmt.js packs the local client's events (localOp / acks / localRollback / localRegen) into the
    same records as streams.py (tests/local_farm.py farms, documents written contiguously; new_ids:
    every reconnect under a new clientId, which keeps short id 0)."""
    from local_farm import replay_log

    log, path = _local_log(tmp_path, new_ids=new_ids)
    script = tmp_path / "local_pack.js"
    script.write_text(_LOCAL_JS % (json.dumps(os.path.join(PKG, "js", "fmt.js")), json.dumps(str(path))) +
                      "const hex=(a)=>Buffer.from(a.buffer,a.byteOffset,a.byteLength).toString('hex');"
                      "process.stdout.write(JSON.stringify({ops:hex(batch.ops),text:hex(batch.text),"
                      "po:Array.from(batch.propsOff),kv:Array.from(batch.propsKv),keys:batch.keys,values:batch.values}));")
    r = _node(str(script))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    py = replay_log(log).finish()
    from fluidframework_amd.streams import MT_F_ACK, MT_F_REGEN, MT_F_ROLLBACK

    f = py.ops["flags"]
    assert ((f & MT_F_ACK) != 0).sum() > 50 and ((f & MT_F_ROLLBACK) != 0).any() and ((f & MT_F_REGEN) != 0).any()
    assert bytes.fromhex(out["ops"]) == py.ops.tobytes()
    assert bytes.fromhex(out["text"]) == py.text.tobytes()
    assert out["po"] == py.props_off.tolist() and out["kv"] == py.props_kv.tolist()
    assert out["keys"] == py.keys and out["values"] == py.values


@pytest.mark.gpu
def test_js_local_client_replay_and_regenerated_ops_on_gpu(addon, orc, tmp_path):
    """The JS driver replays the local farms on the GPU: every participant's local view equals the
    oracle's, and MergeTreeReplay.regenerated(doc) gives the ops the farm resubmitted (the oracle's
    regeneratePendingOp restatement) as IMergeTree*Msg objects."""
    from local_farm import replay_log
    from mt_compare import emu_caps, visible_text

    log, path = _local_log(tmp_path)
    script = tmp_path / "local_gpu.js"
    script.write_text("(async()=>{" + _LOCAL_JS % (json.dumps(os.path.join(PKG, "js", "fmt.js")), json.dumps(str(path))) +
                      "const e=new fmt.Engine(0);const r=await e.replayMergeTree(batch);const out=[];"
                      "for(let d=0;d<batch.nDocs;d++){const h=r.header(d);const segs=h.status===0?r.segments(d):[];"
                      "out.push({status:h.status,text:segs.filter((s)=>s.removedSeq===undefined&&!s.marker)"
                      ".map((s)=>s.text).join(''),regen:r.regenerated(d)});}"
                      "e.close();process.stdout.write(JSON.stringify(out));"
                      "})().catch((e)=>{console.error(e);process.exit(1);});")
    r = _node(str(script), timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    py = replay_log(log).finish()
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(py, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0 and len(got) == py.n_docs
    regen = {}
    for e in log:
        if e[1] == "regen_pending":
            regen.setdefault(e[0], []).extend(e[2])
    n = 0
    for d, g in enumerate(got):
        assert g["status"] == 0, f"doc {d}"
        assert g["text"] == visible_text(oh[d], ol[d], oc[d]), f"doc {d}"
        assert [x["op"] for x in g["regen"]] == regen.get(d, []), f"doc {d}"
        n += len(g["regen"])
    assert n > 10
