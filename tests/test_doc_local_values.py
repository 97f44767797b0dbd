"""Document-local property value ids (fmt.h doc_value_base): a batch whose documents hold more
distinct property values than 16-bit batch-global ids can name (every Marker's unique markerId)
is packed with one dictionary per document instead of being refused (the reference interns no
values at all: properties.ts:68-82, 135-137). Checked through the oracle: each document of the big
batch replays to the same summary as the document packed alone with batch-global ids."""
import numpy as np
import pytest

from marker_docs import marker_batch
from mt_compare import compare_doc

N_DOCS, N_OPS = 200, 1200


def _summary(orc, batch, d):
    return orc.mt_replay_summary(batch, d, batch.keys, batch.doc_values(d))


def test_builder_switches_to_document_local_ids():
    batch = marker_batch(N_DOCS, N_OPS, seed=3)
    assert batch.value_base is not None
    assert len(batch.values) > 65536
    counts = np.diff(batch.value_base.astype(np.int64))
    assert counts.max() < 0xFFFF and counts.min() > 100
    small = marker_batch(4, 200, seed=3)
    assert small.value_base is None  # (a batch that fits keeps batch-global ids)


def test_oracle_document_local_ids_equal_documents_alone(orc):
    batch = marker_batch(N_DOCS, N_OPS, seed=3)
    for d in (0, 1, 77, N_DOCS - 1):
        alone = marker_batch(N_DOCS, N_OPS, seed=3, docs=[d])
        assert alone.value_base is None
        assert _summary(orc, batch, d) == _summary(orc, alone, 0), d
        rc, h1, l1, c1, p1, _ = orc.mt_replay_batch(batch, d, d + 1, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
        rc2, h2, l2, c2, p2, _ = orc.mt_replay_batch(alone, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
        assert rc == 0 and rc2 == 0
        # the same tree and text; prop-set contents differ only by the value numbering
        n = int(h1[0]["n_leaves"])
        assert int(h2[0]["n_leaves"]) == n
        for f in ("ins_seq", "rm_seq", "rm_clients", "len", "block", "pad"):
            assert np.array_equal(l1[0][:n][f], l2[0][:n][f]), f
        assert np.array_equal(c1[0][: int(h1[0]["n_chars"])], c2[0][: int(h2[0]["n_chars"])])


def test_oracle_document_local_ids_with_adjusts(orc):
    """With annotate-adjust the per-document limit is FMT_MT_VALUE_COMPUTED; computed numbers equal
    to a document's own number values take that document's id."""
    batch = marker_batch(120, 900, seed=5, adjust=True)
    assert batch.value_base is not None and batch.adjusts is not None
    for d in (0, 59, 119):
        alone = marker_batch(120, 900, seed=5, adjust=True, docs=[d])
        assert _summary(orc, batch, d) == _summary(orc, alone, 0), d


@pytest.mark.parametrize("adjust", [False, True])
def test_emulated_engine_matches_oracle_on_document_local_ids(orc, adjust):
    from mt_compare import emu_caps, emu_replay
    batch = marker_batch(40, 250, seed=7, adjust=adjust)
    # force local ids on a small batch by building it through the localizing path
    from fluidframework_amd import streams
    b = streams.MergeTreeStreamBuilder()
    import marker_docs
    for d in range(40):
        init, msgs = marker_docs.doc_messages(d, 250, 7, adjust)
        doc = b.begin_doc(init)
        for m in msgs:
            doc.add_message(m)
    b.values.items += [f'"pad{i}"' for i in range(70000 if not adjust else 40000)]  # (unreferenced: only pushes the batch over the limit)
    local = b.finish()
    assert local.value_base is not None and batch.value_base is None
    cl, cc, cp = emu_caps(True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(local, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(local, large=True)
    for d in range(local.n_docs):
        assert compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d])) == [], d
