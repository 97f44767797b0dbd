"""fmt_mt_state_digest on the GPU == the oracle's digest of its own replay, for every document of
batches that cover each place a document's state can live (compact/small-tier slabs, large-tier
slabs, a huge document's own buffers) — the check bench.py runs over the whole T1 batch. A few
documents are also compared field by field, so the digest agreeing means the states agree."""
import numpy as np
import pytest

from fluidframework_amd import native, workloads
from golden_data import replay_fixtures
from mt_compare import compare_doc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = native.Engine(0)
    yield e
    e.close()


def _replay(engine, batch):
    engine.mt_load(batch)
    engine.mt_run()
    hdrs = engine.mt_headers(raise_on_failed_docs=False)
    return hdrs, engine.mt_digests()


def _oracle_digests(orc, batch, threads=16):
    rc, dig, st, _ = orc.mt_replay_digest(batch, threads=threads)
    return rc, dig, st


def test_t1_shape_digests_match_oracle(orc, engine):
    """20k documents of the benchmarked T1 shape (8 writers × 2000 ops): every digest equal."""
    batch = workloads.conflict_farm(20_000, n_clients=8, ops_per_doc=2000, seed=1)
    hdrs, got = _replay(engine, batch)
    assert (hdrs["status"] == 0).all()
    rc, exp, st = _oracle_digests(orc, batch)
    assert rc == 0
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"{len(bad)} documents differ, first {bad[:8].tolist()}"
    cl, cc, cp = native.capacity()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, 0, 8, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    for d in range(8):
        lv, ch, pr = engine.mt_doc(d, hdrs[d])
        assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr))


def test_digests_of_escalated_documents(orc, engine):
    """Long documents (kept >= 3000 units: small tier and large-tier slabs), documents with insert
    props, and enough writers to escalate, in one batch with ordinary ones."""
    long = workloads.conflict_farm(300, n_clients=8, ops_per_doc=1500, min_length=3000, seed=7)
    hdrs, got = _replay(engine, long)
    assert (hdrs["status"] == 0).all()
    rc, exp, _ = _oracle_digests(orc, long)
    assert rc == 0 and np.array_equal(got, exp)
    props = workloads.with_insert_props(workloads.conflict_farm(500, n_clients=40, ops_per_doc=1200, seed=9))
    hdrs, got = _replay(engine, props)
    assert (hdrs["status"] == 0).all()
    rc, exp, _ = _oracle_digests(orc, props)
    assert rc == 0 and np.array_equal(got, exp)


def test_obliterate_farm_digests(orc, engine):
    fixtures = list(replay_fixtures("replay_obliterate_2.3.0.npz"))
    batch = workloads.replicate_batches([f[1] for f in fixtures], 120)
    hdrs, got = _replay(engine, batch)
    assert (hdrs["status"] == 0).all()
    rc, exp, _ = _oracle_digests(orc, batch)
    assert rc == 0 and np.array_equal(got, exp)
    assert np.array_equal(got[:90], np.tile(got[:30], 3))  # copies of one farm digest alike


def test_huge_document_digest(orc, engine):
    """A T3-shaped document (huge tier, its own output buffers)."""
    batch = workloads.t3_stream(200_000, 20_000, n_clients=63, max_lag=4096, max_range=8, seed=3)
    hdrs, got = _replay(engine, batch)
    assert int(hdrs[0]["status"]) == 0
    orc.set_index(True)
    try:
        rc, exp, _ = _oracle_digests(orc, batch, threads=1)
    finally:
        orc.set_index(False)
    assert rc == 0 and int(got[0]) == int(exp[0])


def test_failed_documents_digest_their_status(orc, engine):
    """A document whose replay fails digests (status, fail_seq) only, the same on both sides."""
    batch = workloads.conflict_farm(16, n_clients=8, ops_per_doc=300, seed=11)
    ops = batch.ops
    o = int(batch.doc_op_offsets[5]) + 40
    ops["pos1"][o] = 1_000_000  # past the end: DataProcessingError in the reference
    if int(ops["type"][o]) != 0:  # (an insert's pos2 names its props op)
        ops["pos2"][o] = 1_000_001
    hdrs, got = _replay(engine, batch)
    rc, exp, st = _oracle_digests(orc, batch)
    assert int(hdrs[5]["status"]) == native.FMT_E_DATA and int(st[5]) == native.FMT_E_DATA
    assert np.array_equal(got, exp)
