"""GPU parity: libfmt.so on a real MI355X vs the oracle (bit-exact), through the C ABI.

Run with `pytest -m gpu`. Every comparison is field by field on integer state (no tolerance).
"""
import numpy as np
import pytest

from fluidframework_amd import native, workloads
from fluidframework_amd.streams import MT_OP_DTYPE, MergeTreeBatch
from fluidframework_amd.summary import legacy_summary, map_summary
from golden_data import prefix_batch, replay_fixtures
from mt_compare import compare_doc, visible_text

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = native.Engine(0)
    yield e
    e.close()


def _gpu_mt(engine, batch):
    engine.mt_load(batch)
    engine.mt_run()
    engine.sync()
    hdrs = np.zeros(batch.n_docs, dtype=native.DOC_RESULT_DTYPE)
    import ctypes

    native.lib().fmt_mt_fetch_headers(engine.h, hdrs.ctypes.data_as(ctypes.c_void_p))
    return hdrs


def _check_against_oracle(orc, engine, batch, docs=None):
    hdrs = _gpu_mt(engine, batch)
    cl, cc, cp = native.capacity()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=16, cap_leaves=cl, cap_chars=cc, cap_props=max(cp, 256))
    assert rc == 0
    docs = range(batch.n_docs) if docs is None else docs
    for d in docs:
        leaves, chars, props = engine.mt_doc(d, hdrs[d])
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], leaves, chars, props))
        assert not diffs, f"doc {d}: {diffs[:5]}"
    return hdrs


def test_device_is_gfx950(engine):
    assert "gfx950" in engine.device_info()


def test_map_lww_matches_oracle(orc, engine):
    batch = workloads.map_stream(4000, 1000, key_pool=20, seed=5)
    engine.map_load(batch)
    engine.map_run()
    got = engine.map_fetch()
    exp, _ = orc.map_replay(batch, threads=16)
    assert np.array_equal(got["value"], exp["value"])
    assert np.array_equal(got["birth_seq"], exp["birth_seq"])
    s = engine.stats()
    assert s.ops == len(batch.ops) and s.kernel_ms > 0


def test_map_lww_summaries_match_oracle(orc, engine):
    batch = workloads.map_stream(64, 300, key_pool=20, seed=9)
    engine.map_load(batch)
    engine.map_run()
    got = engine.map_fetch()
    values = [workloads.map_value_json(i) for i in range(50 + 300)]
    small = batch.__class__(batch.ops, batch.doc_op_offsets, batch.key_bound, batch.keys, values)
    for d in range(batch.n_docs):
        assert map_summary(got[d], batch.keys, values) == orc.map_summary(small, d)


def test_map_lww_large_key_pool(orc, engine):
    batch = workloads.map_stream(512, 2000, key_pool=1000, seed=11)
    engine.map_load(batch)
    engine.map_run()
    got = engine.map_fetch()
    exp, _ = orc.map_replay(batch, threads=16)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("n_docs,n_ops,key_pool",
                         [(512, 2000, 1000), (256, 2000, 2560), (256, 2000, 2561), (512, 2000, 5000), (24, 3000, 1 << 20)])
def test_map_lww_key_pool_beyond_lds(orc, engine, n_docs, n_ops, key_pool):
    """Key pools around and over the LDS table's 2560 ids (SURVEY §8d's U[0, 2^20) variant): 2560 ids
    take the LDS kernel with 160 KiB of dynamic LDS per workgroup, 2561 the HBM-table kernels
    (mapLwwHbmKernel + mapLwwFinishKernel); both sides of the switch bit-exact vs the oracle."""
    batch = workloads.map_stream(n_docs, n_ops, key_pool=key_pool, seed=23)
    engine.map_load(batch)
    engine.map_run()
    got = engine.map_fetch()
    exp, _ = orc.map_replay(batch, threads=16)
    assert np.array_equal(got, exp)
    assert int((got["value"] != 0xFFFFFFFF).sum()) > n_docs  # live keys were found
    engine.map_run()  # a second run over the same tables gives the same state
    assert np.array_equal(engine.map_fetch(), exp)


def _dense_to_sparse(exp):
    """Oracle dense slots -> per document [(key, value, birth)] in birth order (JS Map order)."""
    out = []
    for d in range(exp.shape[0]):
        live = np.nonzero(exp["value"][d] != 0xFFFFFFFF)[0]
        rows = sorted((int(exp["birth_seq"][d][k]), int(k), int(exp["value"][d][k])) for k in live)
        out.append([(k, v, b) for b, k, v in rows])
    return out


@pytest.mark.parametrize("n_docs,n_ops,key_pool", [(200, 1000, 20), (64, 1000, 5000), (24, 1000, 1 << 20),
                                                   (16, 1800, 1 << 20), (16, 3000, 1500)])
def test_map_sparse_matches_oracle(orc, engine, n_docs, n_ops, key_pool):
    """Sparse LWW (map_sparse.hip: LDS hash reduce-by-key, one entry per live key in birth order):
    equal to the oracle's dense result, small and 2^20 key pools, register and streaming paths."""
    batch = workloads.map_stream(n_docs, n_ops, key_pool=key_pool, seed=41)
    engine.map_load_sparse(batch)
    engine.map_run_sparse()
    counts, entries = engine.map_fetch_sparse()
    exp, _ = orc.map_replay(batch, threads=16)
    want = _dense_to_sparse(exp)
    assert [len(w) for w in want] == [int(c) for c in counts]
    o = 0
    for d in range(n_docs):
        got = [(int(e["key"]), int(e["value"]), int(e["birth_seq"])) for e in entries[o : o + int(counts[d])]]
        o += int(counts[d])
        assert got == want[d], d
    engine.map_run_sparse()  # a second run gives the same entries
    c2, e2 = engine.map_fetch_sparse()
    assert np.array_equal(c2, counts) and np.array_equal(e2, entries)


def _check_sparse(orc, engine, batch):
    engine.map_load_sparse(batch)
    engine.map_run_sparse()
    counts, entries = engine.map_fetch_sparse()
    wc, we, _ = orc.map_replay_sparse(batch, threads=16)
    assert np.array_equal(counts, wc)
    assert np.array_equal(entries, we)
    return counts


def test_map_sparse_m2_shape_matches_sparse_oracle(orc, engine):
    """The benchmarked shape (1000 ops per document, keys U[0, 2^20)) on 20k documents against the
    sparse oracle, every entry equal; and a 2^20 pool with 200-op documents (smaller tables)."""
    counts = _check_sparse(orc, engine, workloads.map_stream(20000, 1000, key_pool=1 << 20, seed=5))
    assert counts.sum() > 20000
    _check_sparse(orc, engine, workloads.map_stream(5000, 200, key_pool=1 << 20, seed=6))


def test_map_sparse_ragged_documents(orc, engine):
    """Document lengths around every path boundary (0, 1, 63/64/65, 1023/1024/1025 — the register /
    streaming switch — 2048, 4097 and the 16384 maximum) in one batch, small and 2^20 key pools."""
    from fluidframework_amd.streams import MapBatch

    lens = [0, 1, 63, 64, 65, 511, 512, 513, 1023, 1024, 1025, 2048, 4097, 16384, 3, 0, 1000]
    for pool in (20, 3000, 1 << 20):
        src = workloads.map_stream(len(lens), 16384, key_pool=pool, seed=11)
        parts, offs = [], [0]
        for d, n in enumerate(lens):
            o0 = int(src.doc_op_offsets[d])
            parts.append(src.ops[o0 : o0 + n])
            offs.append(offs[-1] + n)
        ops = np.concatenate(parts)
        for d in range(len(lens)):
            ops["doc"][offs[d] : offs[d + 1]] = d
            if lens[d] > 2000:  # at most 2048 distinct keys per document (the table): 1900, spread over the pool
                ops["key"][offs[d] : offs[d + 1]] = ops["key"][offs[d] : offs[d + 1]] % 1900 * max(1, pool // 2000)
        _check_sparse(orc, engine, MapBatch(ops, np.array(offs, dtype=np.uint64), pool, src.keys, src.values))


def test_map_sparse_limits(engine):
    """A key id >= key_bound is FMT_E_DATA; a document with more distinct keys than the table holds
    is FMT_E_CAPACITY (its count 0), the other documents unaffected."""
    from fluidframework_amd.streams import MapBatch

    src = workloads.map_stream(4, 3000, key_pool=1 << 20, seed=43)
    bad = MapBatch(src.ops.copy(), src.doc_op_offsets, 1000, src.keys, src.values)
    engine.map_load_sparse(bad)
    engine.map_run_sparse()
    with pytest.raises(native.EngineError) as ei:
        engine.map_fetch_sparse()
    assert ei.value.code == native.FMT_E_DATA
    # one bad key id before the document's last clear is still FMT_E_DATA (the kernel skips those
    # ops' effects, not their checks): streaming (3000 ops) and register (500 ops) documents
    for n_ops in (3000, 500):
        b2 = workloads.map_stream(4, n_ops, key_pool=1000, seed=44)
        ops = b2.ops.copy()
        ops["kind_value"][10] = 5
        ops["key"][10] = 5000
        ops["kind_value"][20] = 2 << 30
        engine.map_load_sparse(MapBatch(ops, b2.doc_op_offsets, 1000, b2.keys, b2.values))
        engine.map_run_sparse()
        with pytest.raises(native.EngineError) as ei:
            engine.map_fetch_sparse()
        assert ei.value.code == native.FMT_E_DATA
    ops = src.ops.copy()
    o0, o1 = int(src.doc_op_offsets[1]), int(src.doc_op_offsets[2])
    ops["kind_value"][o0:o1] = ops["kind_value"][o0:o1] & 0x3FFFFFFF  # all sets
    ops["key"][o0:o1] = np.arange(o1 - o0, dtype=np.uint32) * 7 + 1   # 3000 distinct keys
    engine.map_load_sparse(MapBatch(ops, src.doc_op_offsets, src.key_bound, src.keys, src.values))
    engine.map_run_sparse()
    with pytest.raises(native.EngineError) as ei:
        engine.map_fetch_sparse()
    assert ei.value.code == native.FMT_E_CAPACITY


def test_mt_bulk_summaries_with_catchup_match_per_document_path(orc, engine):
    """The bulk summary path with catch-up: fmt_mt_summarize_legacy's header/body plus the catchupOps
    blobs from one fmt_mt_fetch_catchup_all copy equal, for every reference replay fixture, the
    per-document path (fetch_doc + Python legacy_summary + fetch_catchup) and the oracle's ranges."""
    from fluidframework_amd import summary
    from test_catchup import fixture_batch

    batch, _ = fixture_batch()
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert (hdrs["status"] == 0).all()
    engine.mt_summarize_legacy(batch.keys, batch.values)
    offs, ranges = engine.mt_catchup_all()
    blobs = summary.bulk_catchup_blobs(batch.messages, hdrs["min_seq"], offs, ranges)
    rc, oh, _, _, _, _, ocu = orc.mt_replay_batch(batch, cap_catchup=4096)
    assert rc == 0
    seen = 0
    for d in range(batch.n_docs):
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert engine.mt_summary(d) == legacy_summary(hdrs[d], lv, ch, pr, batch.keys, batch.values), d
        one = engine.mt_catchup(d, hdrs[d])
        assert np.array_equal(ranges[int(offs[d]) : int(offs[d + 1])], one), d
        assert np.array_equal(one, ocu[d][: int(oh[d]["n_catchup"])]), d
        assert blobs[d] == summary.catchup_blob(summary.catchup_messages(batch.messages[d], one, int(hdrs[d]["min_seq"]))), d
        seen += blobs[d] is not None
    assert seen > 0


def test_map_lww_ragged_documents(orc, engine):
    """Document lengths straddle the register-held path (≤1024 ops) and the streaming path, with
    empty and one-op documents in between."""
    from fluidframework_amd.streams import MapBatch

    src = workloads.map_stream(64, 3000, key_pool=20, seed=13)
    lens = [0, 1, 63, 64, 65, 1000, 1023, 1024, 1025, 2047, 3000, 0, 7, 511, 2999, 128] * 4
    parts, offs = [], [0]
    for d, n in enumerate(lens):
        o = int(src.doc_op_offsets[d])
        p = src.ops[o : o + n].copy()
        p["doc"] = d
        parts.append(p)
        offs.append(offs[-1] + n)
    batch = MapBatch(np.concatenate(parts), np.array(offs, dtype=np.uint64), src.key_bound, src.keys, src.values)
    engine.map_load(batch)
    engine.map_run()
    got = engine.map_fetch()
    exp, _ = orc.map_replay(batch, threads=16)
    assert np.array_equal(got, exp)


def test_mt_reference_fixture_checkpoints(orc, engine):
    """All 30 conflict-farm fixtures × 64 groups: text equals the reference's resultText and the
    whole converged tree equals the oracle's."""
    batch, expected = prefix_batch(list(replay_fixtures()))
    hdrs = _check_against_oracle(orc, engine, batch)
    for d, text in enumerate(expected):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == text, f"doc {d}"


@pytest.mark.parametrize("n_clients,min_length,seed", [(8, 0, 1), (2, 0, 2), (16, 0, 3), (8, 128, 4), (31, 0, 5)])
def test_mt_conflict_farm_matches_oracle(orc, engine, n_clients, min_length, seed):
    batch = workloads.conflict_farm(600, n_clients=n_clients, ops_per_doc=2000, min_length=min_length, seed=seed)
    _check_against_oracle(orc, engine, batch)


@pytest.mark.parametrize("n_clients", [8, 24])
def test_mt_inserts_with_props_match_oracle(orc, engine, n_clients):
    """seg {text, props} inserts (one- and two-key sets, an all-null set): small tier, and with 24
    writers the documents whose prop sets overflow it escalate to the large tier (256 sets)."""
    batch = workloads.with_insert_props(workloads.conflict_farm(64, n_clients=n_clients, ops_per_doc=2000, seed=29))
    hdrs = _check_against_oracle(orc, engine, batch)
    assert (hdrs["status"] == 0).all()


def test_mt_marker_and_props_inserts_match_oracle(orc, engine):
    """Marker inserts and {text, props} inserts (tests/test_insert_props.py's streams) on the GPU."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder
    from test_insert_props import _marker_messages, _messages, _wide_messages

    b = MergeTreeStreamBuilder()
    for msgs in (_messages(), _marker_messages(), _wide_messages(8)):
        d = b.begin_doc("", observer="A")
        for m in msgs:
            d.add_message(m)
    batch = b.finish()
    hdrs = _check_against_oracle(orc, engine, batch)
    assert (hdrs["status"] == 0).all()


def test_mt_summaries_match_oracle(orc, engine):
    batch = workloads.conflict_farm(48, n_clients=8, ops_per_doc=2000, seed=21)
    hdrs = _gpu_mt(engine, batch)
    for d in range(batch.n_docs):
        leaves, chars, props = engine.mt_doc(d, hdrs[d])
        head, body = legacy_summary(hdrs[d], leaves, chars, props, batch.keys, batch.values)
        doc = orc.MergeTreeDoc()
        doc.start_collab(0)
        o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
        doc.apply(batch.ops[o0:o1], batch.text, batch.props_off, batch.props_kv)
        eh, eb = doc.summary(batch.keys, batch.values)
        assert head == eh and body == eb, f"doc {d}"


def test_mt_full_size_properties(orc, engine):
    """T1-shaped batch (20k docs × 2k ops): every doc converges, invariants hold, and a sample
    of documents is bit-exact with the oracle."""
    batch = workloads.conflict_farm(2500, n_clients=8, ops_per_doc=2000, seed=33, replicas=8)
    hdrs = _gpu_mt(engine, batch)
    assert (hdrs["status"] == 0).all()
    assert (hdrs["cur_seq"] == 2000).all()
    # replicas are identical documents in distinct HBM bytes: identical results
    n = 2500
    for f in ("n_leaves", "n_chars", "visible_len", "n_blocks", "min_seq"):
        assert np.array_equal(hdrs[f][:n], hdrs[f][7 * n :])
    sample = list(range(0, batch.n_docs, 997))
    sub = _subset(batch, sample)
    _check_against_oracle(orc, engine, sub)


def _subset(batch, docs):
    ops, offs, init = [], [0], []
    for d in docs:
        o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
        ops.append(batch.ops[o0:o1])
        offs.append(offs[-1] + o1 - o0)
        init.append(batch.doc_init[d])
    return MergeTreeBatch(np.concatenate(ops), np.asarray(offs, np.uint64), batch.text, np.asarray(init, np.uint32),
                          batch.props_off, batch.props_kv, batch.keys, batch.values)


def test_mt_reports_capacity_and_data_errors(engine):
    """Invalid streams fail per document with a status, never crash. A document that overflows the
    small tier replays in the large tier, and past that from its start in the huge tier (no size
    ceiling, test_growth.py)."""
    text = np.full(50000, ord("x"), dtype="<u2")
    ops = np.zeros(4, dtype=MT_OP_DTYPE)
    # doc 0: three inserts totalling 150000 UTF-16 units (> the large tier's 131071: the huge tier)
    ops[0] = (1, 0, 0, 0, -1, 0, 50000, 1, 0, 0)
    ops[1] = (2, 1, 0, 0, -1, 0, 50000, 1, 0, 0)
    ops[2] = (3, 2, 0, 0, -1, 0, 50000, 1, 0, 0)
    # doc 1: insert past the end of an empty document (DataProcessingError)
    ops[3] = (1, 0, 0, 5, -1, 0, 3, 1, 0, 0)
    batch = MergeTreeBatch(ops, np.array([0, 3, 4], np.uint64), text, np.zeros((2, 2), np.uint32),
                           np.zeros(1, np.uint32), np.zeros(0, np.uint32), [], ["null"])
    hdrs = _gpu_mt(engine, batch)
    assert hdrs["status"][0] == native.FMT_OK and hdrs["n_chars"][0] == 150000
    assert hdrs["status"][1] == native.FMT_E_DATA and hdrs["fail_seq"][1] == 1


def test_mt_large_documents_escalate_to_large_tier(orc, engine):
    """Long documents (> 512 leaves or > 2048 UTF-16 units) mixed with ordinary ones: the runtime
    replays the overflowing ones again in the large tier; every document == oracle bit for bit."""
    big = workloads.conflict_farm(24, n_clients=8, ops_per_doc=4000, min_length=3000, seed=21)
    small = workloads.conflict_farm(40, n_clients=8, ops_per_doc=1000, seed=22)
    ops_b = big.ops.copy()
    ins = ops_b["type"] == 0
    ops_b["payload"][ins] += len(small.text)
    init_b = big.doc_init.copy()
    init_b[:, 0] += len(small.text)
    batch = MergeTreeBatch(np.concatenate([small.ops, ops_b]),
                           np.concatenate([small.doc_op_offsets, big.doc_op_offsets[1:] + len(small.ops)]),
                           np.concatenate([small.text, big.text]), np.concatenate([small.doc_init, init_b]),
                           small.props_off, small.props_kv, small.keys, small.values)
    hdrs = _check_against_oracle(orc, engine, batch)
    assert (hdrs["status"] == 0).all()
    assert ((hdrs["n_leaves"] > 512) | (hdrs["n_chars"] > 2048)).sum() >= 12
    assert engine.stats().launches == 3  # compact tier, small tier over its overflow, large tier


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"])
def test_mt_reference_snapshots_load_on_gpu(orc, engine, name):
    """The reference's legacy snapshot fixtures (8.9k-89k chars, up to 1112 segments) load into the
    engine (large tier) and summarize again to the fixture's blobs byte for byte."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder
    from golden_data import snapshot_trees
    from test_oracle_golden import _blobs

    blobs = _blobs(snapshot_trees()[name])
    b = MergeTreeStreamBuilder()
    b.begin_doc_from_summary(blobs["header"], blobs.get("body"))
    batch = b.finish()
    hdrs = _check_against_oracle(orc, engine, batch)
    leaves, chars, props = engine.mt_doc(0, hdrs[0])
    head, body = legacy_summary(hdrs[0], leaves, chars, props, batch.keys, batch.values)
    assert head == blobs["header"] and body == blobs.get("body")


def test_mt_catchup_ranges_match_oracle(orc, engine):
    """Legacy catch-up ranges (FMT_MT_F_CATCHUP ops) bit-exact vs the oracle, and the reload property."""
    from fluidframework_amd import streams, summary
    from test_catchup import CAP, fixture_batch, reload_text

    batch, finals = fixture_batch()
    hdrs = _gpu_mt(engine, batch)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, cap_catchup=CAP)
    assert rc == 0 and (hdrs["status"] == 0).all()
    for d in range(batch.n_docs):
        n = int(oh[d]["n_catchup"])
        got = engine.mt_catchup(d, hdrs[d])
        assert len(got) == n and np.array_equal(got, ocu[d][:n]), d
        leaves, chars, props = engine.mt_doc(d, hdrs[d])
        msgs = summary.catchup_messages(batch.messages[d], got, int(hdrs[d]["min_seq"]))
        assert reload_text(orc, hdrs[d], leaves, chars, props, batch.keys, batch.values, msgs) == finals[d]
    cf = workloads.conflict_farm(512, n_clients=8, ops_per_doc=2000, seed=21)
    streams.flag_catchup(cf.ops, cf.doc_op_offsets)
    hdrs = _gpu_mt(engine, cf)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(cf, threads=16, cap_catchup=CAP)
    assert rc == 0 and (hdrs["status"] == 0).all()
    for d in range(cf.n_docs):
        n = int(oh[d]["n_catchup"])
        assert n > 0 and np.array_equal(engine.mt_catchup(d, hdrs[d]), ocu[d][:n]), d


def test_mt_snapshot_load_matches_oracle(orc, engine):
    """Documents loaded from legacy summaries (+ catch-up ops) replay bit-exactly vs the oracle."""
    from test_catchup import fixture_batch
    from test_snapshot_load import reload_batch, summaries_of

    batch, finals = fixture_batch()
    rb = reload_batch(summaries_of(orc, batch))
    hdrs = _check_against_oracle(orc, engine, rb)
    for d in range(rb.n_docs):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == finals[d]
    cf = workloads.conflict_farm(256, n_clients=8, ops_per_doc=1500, seed=31)
    rb = reload_batch(summaries_of(orc, cf, chunk=60, catchup=False), keep_messages=False)
    _check_against_oracle(orc, engine, rb)


def test_map_split_replay_through_summary(orc, engine):
    """Prefix replay → summary → load + the rest, on the GPU == the oracle's full replay."""
    from test_map_load import split_replay_batches

    full, resumed = split_replay_batches(orc, n_docs=256)
    engine.map_load(resumed)
    engine.map_run()
    got = engine.map_fetch()
    for d in range(full.n_docs):
        assert map_summary(got[d], resumed.keys, resumed.values) == orc.map_summary(full, d), d


def test_mt_obliterate_fixture_checkpoints(orc, engine):
    """f1: all 1920 text checkpoints of the 30 reference obliterate fixtures, engine == oracle."""
    from golden_data import prefix_batch
    from test_obliterate import OB_FIXTURES

    batch, expected = prefix_batch(OB_FIXTURES)
    hdrs = _check_against_oracle(orc, engine, batch)
    for d, text in enumerate(expected):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == text, d


def test_mt_obliterate_farms_through_compact_cascade(orc, engine):
    """The 30 whole obliterate farms, cycled to 600 documents (bench.py --workload ob's batch): the
    compact tier checkpoints the documents that outgrow it, live obliterates included, and the small
    tier resumes them — engine == oracle, final texts == the reference's."""
    from fluidframework_amd.workloads import replicate_batches
    from test_obliterate import OB_FIXTURES

    batch = replicate_batches([f[1] for f in OB_FIXTURES], 600)
    hdrs = _check_against_oracle(orc, engine, batch)
    # compact tier, small tier over its overflow, and the large tier for the few documents that reach
    # the small tier's block / prop-set margins
    assert engine.stats().launches >= 2
    for d in range(len(OB_FIXTURES)):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == OB_FIXTURES[d][4][-1], d


def test_mt_long_obliterate_farms_through_full_cascade(orc, engine):
    """Obliterate documents past the small tier's 6144 units: compact → small → large with both
    checkpoints, the live-obliterate table carried in the compact checkpoint slot — engine == oracle."""
    from test_obliterate import long_obliterate_farms

    batch = long_obliterate_farms()
    hdrs = _check_against_oracle(orc, engine, batch)
    assert (hdrs["status"] == 0).all()
    assert engine.stats().launches == 3  # compact tier, small tier over its overflow, large tier


@pytest.mark.parametrize("rng_seed", [None, 5, 9])
def test_mt_sided_obliterate_on_gpu(orc, engine, rng_seed):
    """Sided obliterate (type 5): the reference obliterate fixtures re-encoded as equivalent sided ops
    reach every text checkpoint (pinned); with exclusive start/end places moved in (rng_seed), engine ==
    oracle bit for bit (parity unpinned: no reference fixture holds an exclusive place)."""
    from golden_data import prefix_batch
    from test_obliterate import OB_FIXTURES
    from test_obliterate_sided import as_sided

    batch, expected = prefix_batch(OB_FIXTURES[::3])
    batch.ops = as_sided(batch.ops, None if rng_seed is None else np.random.default_rng(rng_seed))
    hdrs = _check_against_oracle(orc, engine, batch)
    assert (hdrs["status"] == 0).all()
    if rng_seed is None:
        for d, text in enumerate(expected):
            leaves, chars, _ = engine.mt_doc(d, hdrs[d])
            assert visible_text(hdrs[d], leaves, chars) == text, d


def test_mt_sided_obliterate_catchup_ranges_on_gpu(orc, engine):
    """Catch-up ranges of sided obliterates with exclusive places (OBLITERATE deltas) == oracle."""
    from fluidframework_amd import streams
    from test_obliterate import OB_FIXTURES
    from test_obliterate_sided import as_sided

    cap = 4096
    batch, _ = prefix_batch(OB_FIXTURES[::3])
    batch.ops = as_sided(batch.ops, np.random.default_rng(5))
    streams.flag_catchup(batch.ops, batch.doc_op_offsets)
    hdrs = _gpu_mt(engine, batch)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, threads=16, cap_catchup=cap)
    assert rc == 0 and (hdrs["status"] == 0).all(), np.unique(hdrs["status"])
    obl = 0
    for d in range(batch.n_docs):
        n = int(oh[d]["n_catchup"])
        got = engine.mt_catchup(d, hdrs[d])
        assert len(got) == n and np.array_equal(got, ocu[d][:n]), d
        obl += int((got["type"] == 4).sum())
    assert obl > 0


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"])
def test_mt_v1_fixture_round_trip_on_gpu(orc, engine, name):
    """The reference's SnapshotV1 fixtures load on the GPU (large tier) and summarize again as V1 to
    the fixture's blobs byte for byte."""
    from fluidframework_amd.summary import v1_summary
    from test_snapshot_v1 import _load_v1

    batch, head, bodies = _load_v1(name)
    hdrs = _check_against_oracle(orc, engine, batch)
    leaves, chars, props = engine.mt_doc(0, hdrs[0])
    assert v1_summary(hdrs[0], leaves, chars, props, batch.keys, batch.values, batch.clients[0], {}) == (head, bodies)


def _removers_check(orc, engine, batch, names):
    from fluidframework_amd.summary import NOT_REMOVED, removers_from_engine, v1_summary

    hdrs = _check_against_oracle(orc, engine, batch)
    multi = 0
    for d in range(batch.n_docs):
        leaves, chars, props = engine.mt_doc(d, hdrs[d])
        ops = batch.ops[int(batch.doc_op_offsets[d]) : int(batch.doc_op_offsets[d + 1])]
        got = removers_from_engine(leaves, int(hdrs[d]["n_leaves"]), engine.mt_remove_order(d, hdrs[d]), ops)
        want = orc.mt_removers(batch, d)
        ms = int(hdrs[d]["min_seq"])
        for i in range(int(hdrs[d]["n_leaves"])):
            rm = int(leaves[i]["rm_seq"])
            if rm != NOT_REMOVED and rm > ms:
                assert got.get(i) == want.get(i), (d, i)
                multi += len(want[i]) > 1
        if names is not None:
            assert v1_summary(hdrs[d], leaves, chars, props, batch.keys, batch.values, names(d), got) == \
                v1_summary(hdrs[d], leaves, chars, props, batch.keys, batch.values, names(d), want), d
    return multi


def test_mt_v1_remove_order_on_reference_fixture_messages(orc, engine):
    from test_snapshot_v1 import _collab_batch

    batch = _collab_batch()
    assert _removers_check(orc, engine, batch, lambda d: batch.clients[d]) > 0


def test_mt_v1_remove_order_on_conflict_farm(orc, engine):
    from fluidframework_amd.streams import flag_remove_order

    batch = workloads.conflict_farm(2000, n_clients=8, ops_per_doc=1000, seed=31)
    flag_remove_order(batch.ops, batch.doc_op_offsets)
    assert _removers_check(orc, engine, batch, None) > 0


def test_mt_v1_remove_order_with_obliterates(orc, engine):
    """SnapshotV1 merge info of obliterated segments (movedSeq/movedSeqs/movedClientIds) on the
    reference's obliterate fixture messages: the Ob x Rm engine variant's stamps == the oracle's, and
    the V1 summaries are byte-identical (parity unpinned beyond the oracle, see test_snapshot_v1)."""
    from test_snapshot_v1 import obliterate_v1_batch

    batch = obliterate_v1_batch()
    assert _removers_check(orc, engine, batch, lambda d: batch.clients[d]) > 0


def test_mt_many_writers_escalate_to_large_tier(orc, engine):
    """Documents with up to 63 writers (T3's 64 clients incl. the observer) mixed with ordinary ones:
    the small tier's 31-writer remove-client set overflows and the large tier replays them."""
    many = workloads.conflict_farm(16, n_clients=63, ops_per_doc=1500, seed=13)
    hdrs = _check_against_oracle(orc, engine, many)
    assert (hdrs["status"] == 0).all()
    assert engine.stats().launches == 3  # compact tier, small tier over its overflow, large tier


@pytest.mark.parametrize("key_pool", [20, 5000])
def test_map_replay_device_buffers_and_bad_keys(orc, engine, key_pool):
    """fmt_map_replay_device on torch-owned device buffers equals the staged path; an op whose key
    id is >= key_bound is reported by fmt_map_check (FMT_E_DATA), on both the LDS and the HBM path."""
    import torch

    from fluidframework_amd.native import FMT_E_DATA, MAP_SLOT_DTYPE, EngineError

    batch = workloads.map_stream(64, 600, key_pool=key_pool, seed=31)
    exp, _ = orc.map_replay(batch, threads=16)
    raw = torch.from_numpy(np.ascontiguousarray(batch.ops).view(np.uint8).copy()).cuda()
    offs = torch.from_numpy(np.ascontiguousarray(batch.doc_op_offsets, dtype=np.uint64).view(np.int64).copy()).cuda()
    out = torch.zeros(batch.n_docs * key_pool * 8, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    engine.map_replay_device(raw.data_ptr(), offs.data_ptr(), batch.n_docs, key_pool, out.data_ptr())
    engine.map_check()
    got = out.cpu().numpy().view(MAP_SLOT_DTYPE).reshape(batch.n_docs, key_pool)
    assert np.array_equal(got, exp)
    bad = np.ascontiguousarray(batch.ops).copy()
    bad["key"][5] = key_pool + 3
    bad["kind_value"][5] = 0  # a set
    raw_bad = torch.from_numpy(bad.view(np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    engine.map_replay_device(raw_bad.data_ptr(), offs.data_ptr(), batch.n_docs, key_pool, out.data_ptr())
    with pytest.raises(EngineError) as ei:
        engine.map_check()
    assert ei.value.code == FMT_E_DATA
    if key_pool > 2560:  # the HBM path's u64 view of d_out needs 8-byte alignment
        with pytest.raises(EngineError):
            engine.map_replay_device(raw.data_ptr(), offs.data_ptr(), batch.n_docs, key_pool, out.data_ptr() + 4)


def test_mt_bulk_legacy_summaries_match_host(engine):
    """fmt_mt_summarize_legacy (device extractSync merge + C++ JSON on host threads) equals the
    Python host's legacy_summary of the same state, document by document: conflict farms with
    props inserts (small tier and escalated documents), and the reference snapshots loaded (markers,
    annotations, header + body chunks)."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder
    from golden_data import snapshot_trees
    from test_oracle_golden import _blobs

    batch = workloads.with_insert_props(workloads.conflict_farm(300, n_clients=24, ops_per_doc=2000, seed=47))
    hdrs = _gpu_mt(engine, batch)
    t = engine.mt_summarize_legacy(batch.keys, batch.values)
    assert t["bytes"] > 0
    for d in range(batch.n_docs):
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert engine.mt_summary(d) == legacy_summary(hdrs[d], lv, ch, pr, batch.keys, batch.values), d
    b = MergeTreeStreamBuilder()
    names = ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"]
    blobs = [_blobs(snapshot_trees()[n]) for n in names]
    for bl in blobs:
        b.begin_doc_from_summary(bl["header"], bl.get("body"))
    sb = b.finish()
    _gpu_mt(engine, sb)
    engine.mt_summarize_legacy(sb.keys, sb.values)
    for d, bl in enumerate(blobs):
        assert engine.mt_summary(d) == (bl["header"], bl.get("body")), names[d]


def test_mt_bulk_legacy_summary_of_a_huge_document(orc, engine):
    batch = workloads.t3_stream(100_000, 20_000, n_clients=16, max_lag=512, max_range=8, seed=53)
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    engine.mt_summarize_legacy(batch.keys, batch.values)
    lv, ch, pr = engine.mt_doc(0, hdrs[0])
    assert engine.mt_summary(0) == legacy_summary(hdrs[0], lv, ch, pr, batch.keys, batch.values)


def test_mt_relative_positions_on_gpu(orc, engine):
    """Legacy relativePos1/2 ops (marker-relative positions resolved in the op's perspective): the
    hand cases and generated collaborative streams (markers with their own prop sets, so the runtime
    escalates most of them to the large tier) == the oracle bit for bit."""
    from test_relative_pos import _batch, hand_cases, relative_farm
    from mt_compare import visible_text

    cases = hand_cases()
    batch = _batch(cases)
    hdrs = _check_against_oracle(orc, engine, batch)
    for d, (_, _, want) in enumerate(cases):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == want
    farm, _ = relative_farm()
    hdrs = _check_against_oracle(orc, engine, farm)
    assert (hdrs["status"] == 0).all()


def test_mt_v1_merge_info_load_on_gpu(orc, engine):
    """SnapshotV1 summaries with merge info (mid-stream summaries of the reference's replay fixtures)
    load with their stamps and replay the remaining messages: engine == oracle bit for bit, and the
    final text is the fixture's resultText."""
    from mt_compare import visible_text
    from test_snapshot_v1 import v1_reload_batches

    batch, expected = v1_reload_batches()
    hdrs = _check_against_oracle(orc, engine, batch)
    for d, want in enumerate(expected):
        leaves, chars, _ = engine.mt_doc(d, hdrs[d])
        assert visible_text(hdrs[d], leaves, chars) == want, d


@pytest.mark.parametrize("narrow", [True, False])
def test_mt_annotate_adjust_farms_on_gpu(orc, engine, narrow):
    """Annotate-adjust (computePropertyValue, segmentPropertiesManager.ts:54-78) on the GPU: the
    reference's conflict-farm fixtures with annotates rewritten into adjusts (test_annotate_adjust.py),
    cycled to 120 documents; engine == oracle bit for bit incl. the computed-number tables, final
    texts == the fixtures' resultText. narrow: values stay in the small tier; wide: hundreds of prop
    sets, documents escalate to the large tier."""
    import copy

    from test_annotate_adjust import adjust_fixture_batch

    base, finals = adjust_fixture_batch(narrow=narrow)
    reps = 20
    batch = copy.copy(base)
    n = int(base.doc_op_offsets[-1])
    batch.ops = np.concatenate([base.ops] * reps)
    batch.doc_op_offsets = np.concatenate([base.doc_op_offsets[:-1] + r * n for r in range(reps)] + [[reps * n]]).astype(np.uint64)
    batch.doc_init = np.concatenate([base.doc_init] * reps)
    hdrs = _gpu_mt(engine, batch)
    cl, cc, cp = native.capacity()
    nums = []
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(base, threads=16, cap_leaves=cl, cap_chars=cc, cap_props=max(cp, 256),
                                                numbers=nums)
    assert rc == 0
    computed = 0
    for d in range(batch.n_docs):
        k = d % base.n_docs
        leaves, chars, props = engine.mt_doc(d, hdrs[d])
        diffs = compare_doc((oh[k], ol[k], oc[k], op[k]), (hdrs[d], leaves, chars, props))
        assert not diffs, f"doc {d}: {diffs[:5]}"
        assert np.array_equal(engine.mt_numbers(d), nums[k]), d
        assert visible_text(hdrs[d], leaves, chars) == finals[k]
        computed += len(nums[k])
    assert computed > 0


def test_mt_bulk_legacy_summaries_with_adjusts(orc, engine):
    """fmt_mt_summarize_legacy with computed numbers and getAtSeq(minSeq) (the engine's per-leaf
    PropertiesManager records): every document, adjusts above its final minSeq or not, gives the
    oracle's own SnapshotLegacy bytes (C++ JSON.stringify of the numbers); the Python host over
    fmt_mt_fetch_legacy_props agrees; the hand-worked getAtSeq cases give their stated segments."""
    import json

    from fluidframework_amd.streams import MergeTreeStreamBuilder
    from fluidframework_amd.summary import legacy_summary, values_with_numbers
    from test_annotate_adjust import adjust_fixture_batch, getatseq_cases

    for exact_tail in (True, False):
        batch, _ = adjust_fixture_batch(exact_tail)
        hdrs = _gpu_mt(engine, batch)
        engine.mt_summarize_legacy(batch.keys, batch.values)
        for d in range(batch.n_docs):
            want = orc.mt_replay_summary(batch, d, batch.keys, batch.values)
            assert engine.mt_summary(d) == want, d
            lv, ch, pr = engine.mt_doc(d, hdrs[d])
            vals = values_with_numbers(batch.values, engine.mt_numbers(d))
            got = legacy_summary(hdrs[d], lv, ch, pr, batch.keys, vals, legacy_props=engine.mt_legacy_props(d, hdrs[d]))
            assert got == want, d
    cases = getatseq_cases()
    b = MergeTreeStreamBuilder()
    for init, msgs, _ in cases:
        d = b.begin_doc(init, observer="A")
        for m in msgs:
            d.add_message(m)
    batch = b.finish()
    _gpu_mt(engine, batch)
    engine.mt_summarize_legacy(batch.keys, batch.values)
    for d, (_, _, want) in enumerate(cases):
        assert json.loads(engine.mt_summary(d)[0])["segmentTexts"] == want, d


@pytest.mark.parametrize("adjust", [False, True])
def test_mt_document_local_value_ids_on_gpu(orc, engine, adjust):
    """A batch whose documents hold more distinct property values than batch-global 16-bit ids name
    (each Marker's own markerId; fmt.h doc_value_base): the engine's state == oracle for every
    document, and the runtime's legacy summaries (values looked up per document) == the oracle's."""
    from marker_docs import marker_batch

    batch = marker_batch(200, 1200, seed=3) if not adjust else marker_batch(120, 900, seed=5, adjust=True)
    assert batch.value_base is not None
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert (hdrs["status"] == 0).all()
    engine.mt_summarize_legacy(batch.keys, batch.values)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    assert rc == 0
    for d in range(0, batch.n_docs, 7):
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)) == [], d
        assert engine.mt_summary(d) == orc.mt_replay_summary(batch, d, batch.keys, batch.doc_values(d)), d


def test_mt_wide_prop_sets_on_gpu(orc, engine):
    """20-key formatting runs (prop sets over several records, fmt.h FMT_MT_PROPS_KEYS_MAX) through the
    whole tier cascade == oracle, with their legacy summaries and state digests."""
    from marker_docs import marker_batch

    batch = marker_batch(300, 400, seed=21, wide=20)
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers()
    assert (hdrs["status"] == 0).all()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=8192, cap_chars=1 << 17, cap_props=2048)
    assert rc == 0
    engine.mt_summarize_legacy(batch.keys, batch.values)
    for d in range(0, batch.n_docs, 5):
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)) == [], d
        assert engine.mt_summary(d) == orc.mt_replay_summary(batch, d, batch.keys, batch.doc_values(d)), d
    rc, odig, _, _ = orc.mt_replay_digest(batch, threads=8)
    assert rc == 0
    assert np.array_equal(engine.mt_digests(), odig)
