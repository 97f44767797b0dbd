"""More than 63 writers in one document: short client ids 64..253.

The reference interns client ids without bound (getOrAddShortClientId, client.ts:831-855); a leaf's
remove stamps name any of them (stamps.ts:144-158). The engine's tiers keep remove-client sets of 31
(small), 63 (large) and 253 (huge; 127 until round 6) writers: a document whose ops name an id past
its tier's set grows to the next one, and the huge tier keeps ids 64..253 in a per-leaf-id side
table (huge_engine.h HugeState::hiMask, six words per id) read only by perspectives of those
clients. The ids 64..127 of a leaf's remove-client set are fetched with fmt_mt_fetch_rm_clients_hi,
128..253 with fmt_mt_fetch_rm_clients_hi2, and folded into the state digest under tags 10, 11 and
12. Pins: conflict farms of 96 and 240 writers and T3-shaped documents of 100 and 230 writers,
emulated and on the GPU, equal to the oracle (every leaf field, the text, the prop sets, the ids
64..253 of every remove-client set, the digest)."""
import numpy as np
import pytest

from fluidframework_amd import native, streams, workloads
from digest import state_digest
from mt_compare import compare_doc, emu_huge_replay_hi, oracle_rm_clients_hi, oracle_rm_clients_hi2

CAP_LEAVES, CAP_CHARS, CAP_PROPS = 4096, 8192, 256


def _farm(n_docs=6, n_clients=96, ops=600, seed=11):
    return workloads.conflict_farm(n_docs, n_clients=n_clients, ops_per_doc=ops, seed=seed)


def _t3(n_clients=100, n_ops=2500):
    return workloads.t3_stream(n_segments=3000, n_ops=n_ops, n_clients=n_clients, max_lag=300, seed=4)


def _oracle(orc, batch, cap_leaves=CAP_LEAVES, cap_chars=CAP_CHARS):
    rc, hdrs, leaves, chars, props, _ = orc.mt_replay_batch(batch, cap_leaves=cap_leaves, cap_chars=cap_chars,
                                                            cap_props=CAP_PROPS)
    assert rc == 0
    out = []
    for d in range(batch.n_docs):
        h = hdrs[d]
        n = int(h["n_leaves"])
        out.append((h, leaves[d][:n], chars[d][: int(h["n_chars"])], props[d][: int(h["n_props"])],
                    oracle_rm_clients_hi(batch, d, n), oracle_rm_clients_hi2(batch, d, n)))
    return out


def test_farm_writers_past_63_reach_ids_above_63(orc):
    batch = _farm()
    assert int(batch.ops["client"].max()) > 63
    exp = _oracle(orc, batch)
    assert any(e[4].any() for e in exp), "no leaf holds a remove stamp of a client above 63"


def test_emulated_huge_tier_keeps_127_writers(orc):
    batch = _farm()
    exp = _oracle(orc, batch)
    _, digests, _, _ = orc.mt_replay_digest(batch)
    for d in range(batch.n_docs):
        h, lv, ch, pr, hi = emu_huge_replay_hi(batch, d)
        assert int(h["status"]) == 0
        diffs = compare_doc(exp[d][:4], (h, lv, ch, pr))
        assert not diffs, (d, diffs[:4])
        assert np.array_equal(hi, exp[d][4]), d
        assert state_digest(h, lv, ch, pr, hi) == int(digests[d]), d


def test_emulated_huge_t3_with_100_writers(orc):
    batch = _t3()
    exp = _oracle(orc, batch, cap_leaves=3000 + 3 * 2500 + 8, cap_chars=len(batch.text) + 8)
    h, lv, ch, pr, hi = emu_huge_replay_hi(batch, 0)
    assert int(h["status"]) == 0
    assert not compare_doc(exp[0][:4], (h, lv, ch, pr))
    assert np.array_equal(hi, exp[0][4])
    assert exp[0][4].any()


def test_stream_builder_interns_253_writers():
    b = streams.MergeTreeStreamBuilder()
    d = b.begin_doc()
    for i in range(253):  # every client's stamp stays above minSeq (msn 0): no id can be recycled
        d.add_message({"clientId": f"c{i}", "sequenceNumber": i + 1, "referenceSequenceNumber": 0,
                       "minimumSequenceNumber": 0, "type": "op",
                       "contents": {"type": streams.MT_INSERT, "pos1": 0, "seg": "x"}})
    with pytest.raises(streams.UnsupportedOp):
        d.add_message({"clientId": "one-too-many", "sequenceNumber": 254, "referenceSequenceNumber": 0,
                       "minimumSequenceNumber": 0, "type": "op",
                       "contents": {"type": streams.MT_INSERT, "pos1": 0, "seg": "y"}})


def _emulated_check(orc, batch, **caps):
    exp = _oracle(orc, batch, **caps)
    _, digests, _, _ = orc.mt_replay_digest(batch)
    for d in range(batch.n_docs):
        h, lv, ch, pr, hi, hi2 = emu_huge_replay_hi(batch, d, hi2=True)
        assert int(h["status"]) == 0, (d, int(h["status"]))
        diffs = compare_doc(exp[d][:4], (h, lv, ch, pr))
        assert not diffs, (d, diffs[:4])
        assert np.array_equal(hi, exp[d][4]) and np.array_equal(hi2, exp[d][5]), d
        assert state_digest(h, lv, ch, pr, hi, hi2) == int(digests[d]), d
    return exp


def test_emulated_huge_tier_keeps_240_writers(orc):
    """Twice round 5's ceiling: short ids up to 240 (the side table's words 2..5), remove stamps of
    clients above 127 on many leaves."""
    batch = _farm(n_docs=3, n_clients=240, ops=1200, seed=12)
    assert int(batch.ops["client"].max()) > 200
    exp = _emulated_check(orc, batch)
    assert any(e[5].any() for e in exp), "no leaf holds a remove stamp of a client above 127"


def test_emulated_huge_t3_with_230_writers(orc):
    batch = _t3(n_clients=230, n_ops=4000)
    exp = _emulated_check(orc, batch, cap_leaves=3000 + 3 * 4000 + 8, cap_chars=len(batch.text) + 8)
    assert exp[0][5].any()


def _gpu_check(orc, batch, cap_leaves=CAP_LEAVES, cap_chars=CAP_CHARS):
    exp = _oracle(orc, batch, cap_leaves, cap_chars)
    _, digests, _, _ = orc.mt_replay_digest(batch)
    e = native.Engine(0)
    try:
        e.mt_load(batch)
        e.mt_run()
        hdrs = e.mt_headers(raise_on_failed_docs=False)
        got_digests = e.mt_digests()
        for d in range(batch.n_docs):
            assert int(hdrs[d]["status"]) == 0, (d, int(hdrs[d]["status"]))
            diffs = compare_doc(exp[d][:4], (hdrs[d],) + tuple(e.mt_doc(d, hdrs[d])))
            assert not diffs, (d, diffs[:4])
            assert np.array_equal(e.mt_rm_clients_hi(d, hdrs[d]), exp[d][4]), d
            assert np.array_equal(e.mt_rm_clients_hi2(d, hdrs[d]), exp[d][5]), d
        assert np.array_equal(np.asarray(got_digests, dtype=np.uint64), np.asarray(digests, dtype=np.uint64))
    finally:
        e.close()


@pytest.mark.gpu
def test_farm_of_96_writers_on_gpu(orc):
    _gpu_check(orc, _farm(n_docs=24))


@pytest.mark.gpu
def test_t3_with_100_writers_on_gpu(orc):
    batch = _t3()
    _gpu_check(orc, batch, cap_leaves=3000 + 3 * 2500 + 8, cap_chars=len(batch.text) + 8)


@pytest.mark.gpu
def test_farm_of_240_writers_on_gpu(orc):
    _gpu_check(orc, _farm(n_docs=8, n_clients=240, ops=1200, seed=12))


@pytest.mark.gpu
def test_t3_with_230_writers_on_gpu(orc):
    batch = _t3(n_clients=230, n_ops=4000)
    _gpu_check(orc, batch, cap_leaves=3000 + 3 * 4000 + 8, cap_chars=len(batch.text) + 8)
