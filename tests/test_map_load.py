"""Loading a SharedMap summary and continuing the replay (map side).

SharedMap.loadCore (map/src/map.ts:251-267) → MapKernel.populateFromSerializable
(mapKernel.ts:557-564). Checks: the reference's own summary strings (map.spec.ts:142-317) survive
load → summarize unchanged; and replaying a prefix, summarizing, loading that summary and replaying
the rest gives the same summary as replaying the whole stream (oracle, and the GPU in -m gpu).
"""
import json

import numpy as np
import pytest

from fluidframework_amd import workloads
from fluidframework_amd.streams import MAP_DELETE, MAP_KIND_SHIFT, MAP_SET, MapStreamBuilder

REFERENCE_HEADERS = [
    '{"blobs":[],"content":{"key":{"type":"Plain","value":"value"}}}',
    '{"blobs":[],"content":{"first":{"type":"Plain","value":"second"},"third":{"type":"Plain",'
    '"value":"fourth"},"fifth":{"type":"Plain"},"object":{"type":"Plain","value":{"type":'
    '"__fluid_handle__","url":"/subMap"}}}}',
    '{"blobs":[],"content":{"2":{"type":"Plain","value":4},"10":{"type":"Plain","value":2},'
    '"a":{"type":"Plain","value":3},"b":{"type":"Plain","value":5}}}',
]


@pytest.mark.parametrize("header", REFERENCE_HEADERS)
def test_reference_map_summaries_survive_load(orc, header):
    b = MapStreamBuilder()
    b.begin_doc_from_summary(header)
    assert orc.map_summary(b.finish(), 0)[0] == header


def test_big_map_summary_with_blob_survives_load(orc):
    long = "01234567890"
    for _ in range(12):
        long = long + long
    header = json.dumps({"blobs": ["blob0"], "content": {"key": {"type": "Plain", "value": "value"},
                                                          "zzz": {"type": "Plain", "value": "the end"}}},
                        separators=(",", ":"))
    blob = json.dumps({"longValue": {"type": "Plain", "value": long}}, separators=(",", ":"))
    b = MapStreamBuilder()
    b.begin_doc_from_summary(header, [blob])
    # load order: header content (key, zzz), then blob0 (longValue); summarize re-splits the same way
    assert orc.map_summary(b.finish(), 0) == (header, [blob])


def _messages(batch, d):
    """Back from packed records to map messages (the generator's values are opaque ids)."""
    out = []
    for op in batch.ops[int(batch.doc_op_offsets[d]) : int(batch.doc_op_offsets[d + 1])]:
        kind = int(op["kind_value"]) >> MAP_KIND_SHIFT
        key = batch.keys[int(op["key"])]
        if kind == MAP_SET:
            out.append({"type": "set", "key": key,
                        "value": {"type": "Plain", "value": json.loads(batch.values[int(op["kind_value"]) & 0x3FFFFFFF])}})
        elif kind == MAP_DELETE:
            out.append({"type": "delete", "key": key})
        else:
            out.append({"type": "clear"})
    return out


def split_replay_batches(orc, n_docs=64, n_ops=400, seed=5):
    src = workloads.map_stream(n_docs, n_ops, key_pool=20, seed=seed)
    full, head_b = MapStreamBuilder(), MapStreamBuilder()
    cuts = []
    rng = np.random.default_rng(seed)
    for d in range(n_docs):
        msgs = _messages(src, d)
        cut = int(rng.integers(0, n_ops + 1))
        cuts.append((msgs, cut))
        for b, part in ((full, msgs), (head_b, msgs[:cut])):
            doc = b.begin_doc()
            for i, m in enumerate(part):
                b.add_message(doc, i + 1, m)
    full_batch, head_batch = full.finish(), head_b.finish()
    tail = MapStreamBuilder()
    for d, (msgs, cut) in enumerate(cuts):
        header, blobs = orc.map_summary(head_batch, d)
        doc = tail.begin_doc_from_summary(header, blobs)
        for i, m in enumerate(msgs[cut:]):
            tail.add_message(doc, cut + i + 1, m)
    return full_batch, tail.finish()


def test_split_replay_through_summary_equals_full_replay(orc):
    full, resumed = split_replay_batches(orc)
    for d in range(full.n_docs):
        assert orc.map_summary(resumed, d) == orc.map_summary(full, d), d


@pytest.mark.parametrize("n_docs,n_ops,key_pool", [(64, 1000, 20), (32, 1000, 5000), (16, 1500, 1 << 20)])
def test_sparse_oracle_equals_dense_oracle(orc, n_docs, n_ops, key_pool):
    """The sparse path's oracle (hash-map key index, entries in Map order) equals the dense oracle's
    live slots in birth order: the checker of mapSparseKernel at key pools the dense table cannot hold."""
    batch = workloads.map_stream(n_docs, n_ops, key_pool=key_pool, seed=7)
    exp, _ = orc.map_replay(batch, threads=4)
    counts, entries, _ = orc.map_replay_sparse(batch, threads=4)
    o = 0
    for d in range(n_docs):
        live = np.nonzero(exp["value"][d] != 0xFFFFFFFF)[0]
        want = sorted((int(exp["birth_seq"][d][k]), int(k), int(exp["value"][d][k])) for k in live)
        got = [(int(e["birth_seq"]), int(e["key"]), int(e["value"])) for e in entries[o : o + int(counts[d])]]
        o += int(counts[d])
        assert got == want, d
