"""Obliterate: the reference's 30 `*-conflict-farm-with-obliterate-2.3.0.json` replay
fixtures (merge-tree/src/test/results, replayed by client.replay.spec.ts:20-76 with
mergeTreeEnableObliterate) pin the restatement: every one of the 64 text checkpoints of every file.
"""
import pytest

from golden_data import replay_fixtures

OB_FIXTURES = list(replay_fixtures("replay_obliterate_2.3.0.npz"))


def test_fixtures_hold_obliterates():
    assert len(OB_FIXTURES) == 30
    assert sum(int((b.ops["type"] == 4).sum()) for _, b, *_ in OB_FIXTURES) == 8177


@pytest.mark.parametrize("idx", range(len(OB_FIXTURES)), ids=[f[0] for f in OB_FIXTURES])
def test_oracle_obliterate_fixture_checkpoints(orc, idx):
    name, batch, group_end, initial, results = OB_FIXTURES[idx]
    doc = orc.MergeTreeDoc()
    init = batch.doc_init[0]
    if init[1]:
        doc.insert_local(0, batch.text[init[0] : init[0] + init[1]].tobytes().decode("utf-16-le"))
    doc.start_collab(0)
    start = 0
    for g, end in enumerate(group_end):
        assert doc.text() == initial[g], f"group {g} initial"
        doc.apply(batch.ops[start:end], batch.text, batch.props_off, batch.props_kv)
        assert doc.text() == results[g], f"group {g} result"
        start = end
