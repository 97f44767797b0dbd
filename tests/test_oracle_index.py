"""The oracle's remote-length index (MergeTree::enableIndex, BlockIdx in oracle/mergetree.hpp)
changes nothing but speed: with it on, every replay gives the same headers, leaves, text and prop
sets as the plain subtree sums (which the reference's fixtures pin). It is what lets the oracle
replay T3's single 10M-segment document, as checker and as CPU baseline."""
import numpy as np
import pytest

from fluidframework_amd import workloads
from golden_data import prefix_batch, replay_fixtures


def _both(orc, batch, **kw):
    out = []
    for on in (False, True):
        orc.set_index(on)
        try:
            out.append(orc.mt_replay_batch(batch, threads=8, **kw))
        finally:
            orc.set_index(False)
    return out


def _same(a, b):
    rc0, h0, l0, c0, p0, _ = a
    rc1, h1, l1, c1, p1, _ = b
    assert rc0 == rc1
    assert np.array_equal(h0, h1)
    assert np.array_equal(l0, l1)
    assert np.array_equal(c0, c1)
    assert np.array_equal(p0, p1)


@pytest.mark.parametrize("bundle", ["replay_conflict_farm_0.40.npz", "replay_obliterate_2.3.0.npz"])
def test_index_on_reference_fixture_prefixes(orc, bundle):
    batch, _ = prefix_batch(list(replay_fixtures(bundle)))
    _same(*_both(orc, batch, cap_leaves=2048, cap_chars=8192))


@pytest.mark.parametrize("clients,ops,seed", [(8, 2000, 3), (31, 3000, 5)])
def test_index_on_conflict_farms(orc, clients, ops, seed):
    batch = workloads.conflict_farm(48, n_clients=clients, ops_per_doc=ops, seed=seed)
    _same(*_both(orc, batch, cap_leaves=4096, cap_chars=16384))


@pytest.mark.parametrize("segs,ops,clients,lag", [(3000, 6000, 16, 300), (20000, 20000, 63, 4096)])
def test_index_on_t3_shaped_documents(orc, segs, ops, clients, lag):
    batch = workloads.t3_stream(segs, ops, n_clients=clients, max_lag=lag, seed=11)
    a, b = _both(orc, batch, cap_leaves=segs + 3 * ops, cap_chars=segs * 8 + ops * 3)
    assert a[0] == 0 and int(a[1]["status"][0]) == 0
    _same(a, b)
