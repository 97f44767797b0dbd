"""More live obliterates than a register tier's table holds (Obliterates, mergeTree.ts:515-635).

Every obliterate above minSeq stays in Obliterates.seqOrdered / startOrdered until minSeq passes it.
The compact / small / large tiers hold 64 in LDS; a document with more escalates (FMT_E_CAPACITY) to
the huge tier, whose table lives in HBM (huge_engine.h HugeState::obRec / obSeq / obStart: one slot
per obliterate op of the document). Pins: documents with 200-300 obliterates that all stay live
(every op references seq 0 and msn stays 0) from 8 clients, with concurrent inserts landing inside
them (obliterate-on-insert), emulated huge tier and GPU == oracle."""
import random

import pytest

from fluidframework_amd import native
from fluidframework_amd.streams import MT_INSERT, MT_OBLITERATE, MergeTreeStreamBuilder
from mt_compare import compare_doc, emu_huge_replay


def _doc(b, seed, n_ops, init_len=3000, n_clients=8):
    rnd = random.Random(seed)
    init = "".join(chr(ord("a") + rnd.randrange(26)) for _ in range(init_len))
    d = b.begin_doc(init, observer="observer")
    view = {c: init_len for c in range(n_clients)}  # each client's own view at refSeq 0
    n_ob = 0
    for k in range(n_ops):
        c = rnd.randrange(n_clients)
        if rnd.random() < 0.8 and view[c] > 4:
            a = rnd.randrange(view[c] - 3)
            n = rnd.randint(1, 3)
            op = {"type": MT_OBLITERATE, "pos1": a, "pos2": a + n}
            view[c] -= n
            n_ob += 1
        else:
            s = "XYZ"[: rnd.randint(1, 3)]
            op = {"type": MT_INSERT, "pos1": rnd.randrange(view[c] + 1), "seg": s}
            view[c] += len(s)
        d.add_message({"clientId": f"w{c}", "sequenceNumber": k + 1, "referenceSequenceNumber": 0,
                       "minimumSequenceNumber": 0, "type": "op", "contents": op})
    return n_ob


def _batch(sizes=(260, 320, 300), seed=3):
    b = MergeTreeStreamBuilder()
    n_ob = [_doc(b, seed + i, n) for i, n in enumerate(sizes)]
    return b.finish(), n_ob


def _oracle(orc, batch):
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=8192, cap_chars=1 << 14, cap_props=64)
    assert rc == 0
    return [(oh[d], ol[d][: int(oh[d]["n_leaves"])], oc[d][: int(oh[d]["n_chars"])], op[d][: int(oh[d]["n_props"])])
            for d in range(batch.n_docs)]


def test_documents_keep_200_live_obliterates(orc):
    batch, n_ob = _batch()
    assert min(n_ob) >= 200
    exp = _oracle(orc, batch)
    assert all(int(e[0]["min_seq"]) == 0 for e in exp)  # (none left the collab window)


def test_emulated_huge_tier_holds_200_live_obliterates(orc):
    batch, _ = _batch()
    exp = _oracle(orc, batch)
    for d in range(batch.n_docs):
        got = emu_huge_replay(batch, d)
        assert int(got[0]["status"]) == 0
        assert compare_doc(exp[d], got) == [], d


@pytest.mark.gpu
def test_200_live_obliterates_on_gpu(orc):
    """The register tiers' 64-entry tables overflow; the documents grow to the huge tier == oracle."""
    batch, _ = _batch()
    exp = _oracle(orc, batch)
    eng = native.Engine(0)
    try:
        eng.mt_load(batch)
        eng.mt_run()
        hdrs = eng.mt_headers()
        for d in range(batch.n_docs):
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            assert compare_doc(exp[d], (hdrs[d], lv, ch, pr)) == [], d
            assert eng.huge_profile(d)["replay"] > 0  # (it ran in the huge tier)
    finally:
        eng.close()
