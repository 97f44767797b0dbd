"""No document-size ceiling: a document that outgrows the large tier (2048 leaves,
131,071 UTF-16 units, 1023 blocks, 1024 prop sets) replays again from its start in the huge tier
(runtime.cpp: the large tier's FMT_E_CAPACITY documents; huge_engine.h from an empty document or its
initial text), as the reference grows its tree without bound (insertSegments, mergeTree.ts:1484-1517).

CPU: the emulated huge tier from an empty start and from an initial text == the oracle bit for bit,
with its index invariants checked after every op. GPU (-m gpu): through the C ABI, documents that grow
past the large tier's limits are escalated and equal the oracle; ordinary documents of the same batch
are unaffected.
"""
import numpy as np
import pytest

from growth import growth_batch
from mt_compare import compare_doc, emu_huge_replay


def _oracle(orc, batch):
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=4096)
    assert rc == 0
    return oh, ol, oc, op


@pytest.mark.parametrize("initial,n_ops,seed", [("", 1500, 1), ("abc" * 300, 1500, 2)])
def test_emulated_huge_tier_from_empty_and_initial_text(orc, initial, n_ops, seed):
    batch = growth_batch([(initial, n_ops, seed)])
    oh, ol, oc, op = _oracle(orc, batch)
    h, lv, ch, pr = emu_huge_replay(batch, 0)
    assert h["status"] == 0
    assert not compare_doc((oh[0], ol[0], oc[0], op[0]), (h, lv, ch, pr))


@pytest.mark.gpu
def test_documents_grow_past_the_large_tier_on_gpu(orc):
    """Two documents that grow from empty / a short initial text past 131,071 UTF-16 units, between
    ordinary conflict-farm documents: the large tier reports them full, the huge tier replays them
    from the start, and every document equals the oracle."""
    from fluidframework_amd import native

    big = growth_batch([("", 6000, 11), ("xyz" * 100, 6000, 12)])
    oh, ol, oc, op = _oracle(orc, big)
    assert (oh["n_chars"] > 131071).all()
    eng = native.Engine(0)
    try:
        eng.mt_load(big)
        eng.mt_run()
        hdrs = eng.mt_headers()
        assert (hdrs["status"] == 0).all(), hdrs["status"]
        assert eng.stats().launches == 4  # compact, small, large, then the huge-tier pass
        for d in range(big.n_docs):
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdrs[d], lv, ch, pr)), d
        eng.mt_run()  # a second run escalates them again, from the start
        assert (eng.mt_headers()["n_chars"] == oh["n_chars"]).all()
    finally:
        eng.close()
