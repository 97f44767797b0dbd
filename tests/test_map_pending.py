"""SharedMap's local-client pending state (map half): MapKernel.pendingData
(mapKernel.ts:132-139) built by local set / delete / clear (:388-538), emptied by acks (the
handlers' local branches, :706-853) and rollbacks (:633-700), read through get() and the
optimistic iterator (:176-240, :374-392). The oracle (oracle/map.cpp PendingMap) is pinned by the
scenarios the reference's own tests assert (tests/golden/map_pending_cases.json, transcribed from
map.rollback.spec.ts and map.iteration.spec.ts); the device path (csrc/map_pending.hip,
fmt_map_pending_run) is compared with the oracle on those and on generated local/remote farms."""
import json
import os
import random

import numpy as np
import pytest

from fluidframework_amd.streams import MAP_EV_ACK, MAP_EV_ROLLBACK, MAP_PENDING_BIRTH, MapStreamBuilder

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "map_pending_cases.json")


def _plain(op):
    if op["type"] != "set":
        return op
    return {"type": "set", "key": op["key"], "value": {"type": "Plain", "value": op["value"]}}


def golden_checkpoints():
    """(builder, [(doc, case index, assertion)]): one document per assertion of each case, holding
    the case's steps up to it."""
    cases = json.load(open(GOLDEN))["cases"]
    b = MapStreamBuilder()
    checks = []
    for ci, case in enumerate(cases):
        for si, step in enumerate(case["steps"]):
            if not step[0].startswith("expect"):
                continue
            d = b.begin_doc()
            seq = 0
            for st in case["steps"][:si]:
                if st[0] == "local":
                    b.local_submit(d, _plain(st[1]))
                elif st[0] == "flush":
                    while b._unacked[d]:
                        seq += 1
                        b.local_ack(d, seq)
                elif st[0] == "remote":
                    seq += 1
                    b.add_message(d, seq, _plain(st[1]))
                elif st[0] == "rollback_all":
                    while b._unacked[d]:
                        b.local_rollback(d)
            checks.append((d, ci, step))
    return b, checks


def _views(batch, counts, entries):
    out, at = [], 0
    for d in range(batch.n_docs):
        n = int(counts[d])
        out.append([(batch.keys[int(e["key"])], json.loads(batch.values[int(e["value"])]))
                    for e in entries[at: at + n]])
        at += n
    return out


def _check_assertion(view, step):
    kind, want = step
    if kind == "expect":
        assert view == [tuple(x) for x in want]
    elif kind == "expect_keys":
        assert [k for k, _ in view] == want
    else:  # expect_get: get(key) per key (null: undefined)
        got = dict(view)
        for k, v in want.items():
            assert got.get(k) == v, (k, got)


def test_oracle_matches_reference_scenarios(orc):
    b, checks = golden_checkpoints()
    batch = b.finish()
    counts, status, entries = orc.map_pending(batch)
    assert (status == 0).all()
    views = _views(batch, counts, entries)
    for d, ci, step in checks:
        _check_assertion(views[d], step)


def test_builder_records_events_in_order():
    b = MapStreamBuilder()
    d = b.begin_doc()
    b.local_submit(d, _plain({"type": "set", "key": "a", "value": 1}))
    b.local_submit(d, {"type": "clear"})
    b.local_ack(d, 1)
    b.local_rollback(d)
    batch = b.finish()
    assert list(batch.local_ops["event"]) == [0, 0, MAP_EV_ACK, MAP_EV_ROLLBACK]
    assert list(batch.local_offsets) == [0, 4]
    assert len(batch.ops) == 1  # (the acknowledged set is sequenced)
    with pytest.raises(ValueError):
        b.local_rollback(d)


def pending_farm(n_docs, n_steps, seed=1, n_keys=6, bad_every=0):
    """Generated local/remote interleavings: the local client submits, gets acks in order, rolls
    back its newest op; a remote client's ops are sequenced between. Documents end with ops still
    pending. bad_every > 0: every such document gets an ACK whose op differs from the oldest
    pending one (the reference asserts: FMT_E_DATA)."""
    rnd = random.Random(seed)
    b = MapStreamBuilder()
    for d in range(n_docs):
        doc = b.begin_doc()
        seq = 0

        def op():
            r = rnd.random()
            k = f"k{rnd.randrange(n_keys)}"
            if r < 0.6:
                return _plain({"type": "set", "key": k, "value": rnd.randrange(50)})
            if r < 0.9:
                return {"type": "delete", "key": k}
            return {"type": "clear"}
        for _ in range(n_steps):
            r = rnd.random()
            if r < 0.45:
                b.local_submit(doc, op())
            elif r < 0.65 and b._unacked[doc]:
                seq += 1
                b.local_ack(doc, seq)
            elif r < 0.75 and b._unacked[doc]:
                b.local_rollback(doc)
            else:
                seq += 1
                b.add_message(doc, seq, op())
        if bad_every and d % bad_every == 0:
            b.local_submit(doc, _plain({"type": "set", "key": "k0", "value": 1}))
            key = b.keys.intern("k0")
            b.local[doc].append((doc, key, MAP_EV_ACK, 0x3FFFFFFE))  # (a value no submission holds)
    return b.finish()


def test_oracle_farm_statuses(orc):
    batch = pending_farm(60, 80, seed=2, bad_every=7)
    counts, status, entries = orc.map_pending(batch)
    assert set(status[::7].tolist()) == {-2}
    assert (np.delete(status, np.arange(0, 60, 7)) == 0).all()
    assert (entries["birth_seq"] & MAP_PENDING_BIRTH != 0).any()  # pending lifetimes iterate
    assert (entries["birth_seq"] & MAP_PENDING_BIRTH == 0).any()


@pytest.mark.gpu
def test_pending_view_on_gpu_matches_oracle_and_reference_scenarios(orc):
    from fluidframework_amd import native
    b, checks = golden_checkpoints()
    batch = b.finish()
    farm = pending_farm(4000, 120, seed=3, bad_every=11)
    e = native.Engine(0)
    try:
        for bt in (batch, farm):
            e.map_load_sparse(bt)
            e.map_run_sparse()
            got = e.map_pending(bt)
            exp = orc.map_pending(bt)
            assert np.array_equal(got[1], exp[1])
            assert np.array_equal(got[0], exp[0])
            assert np.array_equal(got[2], exp[2])
            views = _views(bt, got[0], got[2])
            if bt is batch:
                for d, ci, step in checks:
                    _check_assertion(views[d], step)
    finally:
        e.close()


@pytest.mark.gpu
def test_pending_event_cap_per_document(orc):
    """FMT_MAP_PENDING_MAX_EVENTS: a document with exactly the cap of local events replays (its view
    equals the oracle's); one past it gets FMT_E_CAPACITY and no entries, its neighbours unaffected."""
    from fluidframework_amd import native
    cap = native.MAP_PENDING_MAX_EVENTS
    b = MapStreamBuilder()
    for n in (cap, cap + 1, 10):
        d = b.begin_doc()
        seq = 0
        for i in range(n):
            if i % 2 == 0 or not b._unacked[d]:
                b.local_submit(d, _plain({"type": "set", "key": f"k{i % 5}", "value": i % 50}))
            else:
                seq += 1
                b.local_ack(d, seq)
    bt = b.finish()
    assert list(np.diff(bt.local_offsets)) == [cap, cap + 1, 10]
    e = native.Engine(0)
    try:
        e.map_load_sparse(bt)
        e.map_run_sparse()
        counts, status, entries = e.map_pending(bt)
    finally:
        e.close()
    exp = orc.map_pending(bt)
    assert list(status) == [0, -3, 0]
    assert counts[1] == 0
    assert counts[0] == exp[0][0] and counts[2] == exp[0][2]
    off = np.concatenate([[0], np.cumsum(counts, dtype=np.int64)])
    eoff = np.concatenate([[0], np.cumsum(exp[0], dtype=np.int64)])
    for d in (0, 2):
        assert np.array_equal(entries[off[d]:off[d + 1]], exp[2][eoff[d]:eoff[d + 1]])
