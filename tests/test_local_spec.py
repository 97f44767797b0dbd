"""The reference's local-client spec cases (client.rollback.spec.ts, client.applyMsg.spec.ts,
resetPendingSegmentsToOp.spec.ts), transcribed as data in tests/golden/local_spec_cases.json and run
by tests/local_spec.py: every assertion the specs make on replay state, checked on the oracle, the
emulated engine (CPU) and libfmt.so (GPU)."""
import pytest

from local_spec import evaluate, load_cases, spec_batch
from mt_compare import compare_doc, emu_caps, emu_regen, emu_replay_local


@pytest.fixture(scope="module")
def specs():
    return spec_batch()


def _results(hdr, leaves, chars, props):
    return [(hdr[d], leaves[d][: int(hdr[d]["n_leaves"])], chars[d], props[d]) for d in range(len(hdr))]


def _oracle(orc, batch):
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    return oh, ol, oc, op


def test_spec_cases_are_transcribed(specs):
    cases = load_cases()
    assert len(cases) >= 55
    batch, where = specs
    assert len({w[0] for w in where}) == len(cases)  # every case has a checkpoint


def test_oracle_meets_the_spec_assertions(orc, specs):
    batch, where = specs
    out = _oracle(orc, batch)
    fails = evaluate(batch, where, _results(*out), lambda d: orc.mt_replay_regen(batch, d)[1:])
    assert not fails, fails[:10]


def test_emulated_engine_meets_the_spec_assertions_and_matches_the_oracle(orc, specs):
    batch, where = specs
    got = emu_replay_local(batch)
    fails = evaluate(batch, where, _results(*got), emu_regen)
    assert not fails, fails[:10]
    oh, ol, oc, op = _oracle(orc, batch)
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (got[0][d], got[1][d], got[2][d], got[3][d]))
        assert not diffs, f"{where[d][:2]} step {where[d][3]}: {diffs[:4]}"


@pytest.mark.gpu
def test_gpu_meets_the_spec_assertions_and_matches_the_oracle(orc, specs):
    import numpy as np

    from fluidframework_amd import native

    batch, where = specs
    e = native.Engine(0)
    try:
        e.mt_load(batch)
        e.mt_run()
        e.sync()
        hdr = e.mt_headers(raise_on_failed_docs=False)
        res = []
        for d in range(batch.n_docs):
            leaves, chars, props = e.mt_doc(d, hdr[d])
            res.append((hdr[d], leaves, chars, props))
        regen = [e.mt_regen(d) for d in range(batch.n_docs)]
    finally:
        e.close()
    fails = evaluate(batch, where, res, lambda d: regen[d])
    assert not fails, fails[:10]
    oh, ol, oc, op = _oracle(orc, batch)
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), res[d])
        assert not diffs, f"{where[d][:2]} step {where[d][3]}: {diffs[:4]}"
        o_ops = orc.mt_replay_regen(batch, d)[1]
        assert np.array_equal(o_ops, regen[d][0]), f"{where[d][:2]}: regenerated ops differ"
