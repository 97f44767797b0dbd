"""The merge-tree engine source (mt_engine.h) under host emulation vs the oracle (CPU only).

The same source is compiled into the gfx950 kernel; these tests pin its algorithm before a GPU is
involved. The GPU tests (test_gpu_parity.py) then repeat the comparison on the device.
"""
import numpy as np
import pytest

from fluidframework_amd import workloads
from golden_data import prefix_batch, replay_fixtures
from mt_compare import compare_doc, emu_caps, emu_replay, visible_text


@pytest.fixture(scope="module")
def fixtures_prefix():
    return prefix_batch(list(replay_fixtures()))


def test_emulated_engine_matches_reference_text_checkpoints(fixtures_prefix):
    batch, expected = fixtures_prefix
    hdr, leaves, chars, props = emu_replay(batch)
    assert (hdr["status"] == 0).all(), np.unique(hdr["status"])
    for d, text in enumerate(expected):
        assert visible_text(hdr[d], leaves[d], chars[d]) == text, f"doc {d}"


def test_emulated_engine_matches_oracle_on_fixtures(orc, fixtures_prefix):
    batch, _ = fixtures_prefix
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch)
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


@pytest.mark.parametrize("n_clients,min_length", [(8, 0), (3, 0), (16, 0), (8, 64)])
def test_emulated_engine_matches_oracle_on_conflict_farm(orc, n_clients, min_length):
    batch = workloads.conflict_farm(40, n_clients=n_clients, ops_per_doc=1500, min_length=min_length, seed=7)
    cl, cc, cp = emu_caps()
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch)
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def _no_zamboni_batch(sizes, seed=11):
    """One client inserting 2-char runs at random visible positions with minSeq pinned at 0, so no
    leaf is ever merged or dropped: leaf counts climb through every register row to capacity."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    rng = np.random.default_rng(seed)
    b = MergeTreeStreamBuilder()
    for n_ops in sizes:
        d = b.begin_doc()
        length = 0
        for k in range(n_ops):
            seq = k + 1
            if k % 7 == 6 and length > 4:  # some removes and annotates in the mix
                a = int(rng.integers(0, length - 2))
                contents = {"type": 1, "pos1": a, "pos2": a + 1} if k % 2 else \
                    {"type": 2, "pos1": a, "pos2": a + 2, "props": {"k": int(k % 3)}}
                if k % 2:
                    length -= 1
            else:
                contents = {"type": 0, "pos1": int(rng.integers(0, length + 1)), "seg": "xy"}
                length += 2
            d.add_message({"clientId": "B", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                           "minimumSequenceNumber": 0, "contents": contents})
    return b.finish()


def test_emulated_engine_fills_every_row_to_capacity(orc):
    cl, cc, cp = emu_caps()
    batch = _no_zamboni_batch([60, 130, 200, 260, 300, 400, 420, 500])
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=4, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch)
    assert oh["n_leaves"].max() > cl  # the last documents overflow the 512-leaf engine
    assert ((oh["n_leaves"] > 448) & (oh["n_leaves"] <= cl)).any()  # and one ends in the top row
    for d in range(batch.n_docs):
        if oh[d]["n_leaves"] > cl:
            assert hdr[d]["status"] == -3, f"doc {d}: expected FMT_E_CAPACITY"
            continue
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


# ---- compact tier (4 register rows: plain batches start in it, on the GPU) --------------------------

@pytest.mark.parametrize("n_clients", [8, 3])
def test_compact_tier_matches_oracle_on_conflict_farm(orc, n_clients):
    """The 4-row compact tier is the same engine source: bit-exact vs the oracle on T1-shaped
    documents; a document it cannot hold reports FMT_E_CAPACITY (the runtime then replays it in the
    small tier)."""
    batch = workloads.conflict_farm(40, n_clients=n_clients, ops_per_doc=1500, seed=17)
    cl, cc, cp = emu_caps(large=2)
    assert cl == 256
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=4096, cap_chars=cc, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=2)
    fit = 0
    for d in range(batch.n_docs):
        if hdr[d]["status"] == -3:
            continue
        fit += 1
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
    assert fit >= 30


@pytest.mark.parametrize("n_clients,seed", [(8, 1), (3, 2), (16, 3)])
def test_compact_to_small_cascade_resumes_from_checkpoints(orc, n_clients, seed):
    """The runtime's cascade for plain batches: the compact tier stops a document before the op that
    could outgrow its 256 leaves and saves its state; the small tier resumes it from that op. Every
    document == oracle bit for bit, and checkpoints were taken."""
    batch = workloads.conflict_farm(120, n_clients=n_clients, ops_per_doc=2000, seed=seed)
    cl, cc, cp = emu_caps(large=3)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    compact = emu_replay(batch, large=2)[0]
    assert (compact["status"] == -3).sum() >= 5  # documents that outgrow the compact rows
    hdr, leaves, chars, props = emu_replay(batch, large=3)
    assert (hdr["status"] == 0).all()
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_compact_cascade_checkpoints_long_texts(orc):
    """Documents kept above 3000 UTF-16 units: the compact tier (2048 units) checkpoints before the
    insert that would outgrow its text, and the small tier (6144 units) resumes them."""
    batch = workloads.conflict_farm(24, n_clients=8, ops_per_doc=2000, min_length=3000, seed=21)
    cl, cc, cp = emu_caps(large=3)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=3)
    fits = (oh["n_leaves"] <= cl) & (oh["n_chars"] <= cc)
    assert (oh["n_chars"][fits] > 2048).sum() >= 5, oh["n_chars"][fits]
    for d in range(batch.n_docs):
        if hdr[d]["status"] in (-3, -34):  # beyond the small tier too (the runtime's large tier takes it)
            continue
        assert hdr[d]["status"] == 0
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


@pytest.mark.parametrize("n_clients,min_length,n_ops", [(8, 3000, 2000), (40, 0, 1500)])
def test_full_cascade_resumes_in_the_large_tier(orc, n_clients, min_length, n_ops):
    """compact → small → large with checkpoints: documents past 512 leaves, 6144 units or 31
    writers leave the small tier at an op boundary and the large tier converts its state (W0 packing,
    8-bit block ids, text into the HBM slab) and resumes them; every document == oracle."""
    batch = workloads.conflict_farm(24, n_clients=n_clients, ops_per_doc=n_ops, min_length=min_length, seed=33)
    cl, cc, cp = emu_caps(large=4)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    small = emu_replay(batch, large=3)[0]
    assert (small["status"] == -34).sum() >= 2  # checkpointed for the large tier
    hdr, leaves, chars, props = emu_replay(batch, large=4)
    assert (hdr["status"] == 0).all(), hdr["status"]
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_compact_cascade_with_catchup_and_props(orc):
    """Checkpointed documents keep their catch-up ranges (recorded before and after the checkpoint)
    and prop sets."""
    from fluidframework_amd.streams import flag_catchup

    batch = workloads.conflict_farm(60, n_clients=8, ops_per_doc=2000, seed=9)
    flag_catchup(batch.ops, batch.doc_op_offsets)
    cl, cc, cp = emu_caps(large=3)
    rc, oh, ol, oc, op, _, ocu = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024,
                                                     cap_catchup=4096)
    assert rc == 0
    hdr, leaves, chars, props, cu = emu_replay(batch, large=3, cap_catchup=4096)
    assert (hdr["status"] == 0).all()
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
        n = int(oh[d]["n_catchup"])
        assert int(hdr[d]["n_catchup"]) == n and np.array_equal(cu[d][:n], ocu[d][:n]), d


def test_compact_tier_fills_every_row_to_capacity(orc):
    cl, cc, cp = emu_caps(large=2)
    batch = _no_zamboni_batch([60, 130, 200, 230, 250, 260, 300])
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=4, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=2)
    assert oh["n_leaves"].max() > cl and ((oh["n_leaves"] > 192) & (oh["n_leaves"] <= cl)).any()
    for d in range(batch.n_docs):
        if oh[d]["n_leaves"] > cl:
            assert hdr[d]["status"] == -3, f"doc {d}: expected FMT_E_CAPACITY"
            continue
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


# ---- large tier (documents that overflow the small tier replay again in it, on the GPU) ----------

def test_large_tier_matches_oracle_on_fixtures(orc, fixtures_prefix):
    """The rolled, HBM-text large tier is the same engine: bit-exact vs the oracle where both fit."""
    batch, expected = fixtures_prefix
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        assert visible_text(hdr[d], leaves[d], chars[d]) == expected[d], f"doc {d}"
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_large_tier_fills_every_row_to_capacity(orc):
    """Documents of 600..2300 leaves: beyond the small tier's 512, up to and past the large tier's 2048."""
    cl, cc, cp = emu_caps(large=True)
    small_leaves = emu_caps()[0]
    batch = _no_zamboni_batch([400, 1000, 1500, 1650, 1800], seed=5)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=4, cap_leaves=8192, cap_chars=1 << 17, cap_props=1024)
    assert rc == 0
    assert oh["n_leaves"].max() > cl and ((oh["n_leaves"] > small_leaves) & (oh["n_leaves"] <= cl)).sum() >= 2
    small = emu_replay(batch)[0]
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        if oh[d]["n_leaves"] > small_leaves:
            assert small[d]["status"] == -3, f"doc {d}: the small tier must overflow"
        if oh[d]["n_leaves"] > cl:
            assert hdr[d]["status"] == -3, f"doc {d}: expected FMT_E_CAPACITY"
            continue
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_large_tier_matches_oracle_on_long_conflict_farm(orc):
    """Conflict-farm documents long enough to outgrow 2048 UTF-16 units / 512 leaves."""
    batch = workloads.conflict_farm(6, n_clients=8, ops_per_doc=4000, min_length=3000, seed=21)
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=6, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    small_cl, small_cc, _ = emu_caps()
    assert ((oh["n_leaves"] > small_cl) | (oh["n_chars"] > small_cc)).any()
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_emulated_engine_newline_segments_stop_appends(orc):
    """Zamboni appends stop after a segment ending in '\\n' (TextSegment.canAppend,
    textSegment.ts:76-93); texts with newlines, acked at once (minSeq = seq - 1), both tiers."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    rng = np.random.default_rng(3)
    b = MergeTreeStreamBuilder()
    pieces = ["a\n", "bc", "\n", "xyz\n", "q", "rs", "\nt"]
    for doc in range(6):
        d = b.begin_doc()
        length = 0
        for k in range(300):
            seq = k + 1
            if k % 5 == 4 and length > 3:
                a = int(rng.integers(0, length - 1))
                contents = {"type": 1, "pos1": a, "pos2": a + 1}
                length -= 1
            else:
                t = pieces[int(rng.integers(0, len(pieces)))]
                contents = {"type": 0, "pos1": int(rng.integers(0, length + 1)), "seg": t}
                length += len(t)
            d.add_message({"clientId": "BC"[k % 2], "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
                           "minimumSequenceNumber": max(0, seq - 1 - doc), "contents": contents})
    batch = b.finish()
    for large in (False, True):
        cl, cc, cp = emu_caps(large)
        rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=4, cap_leaves=cl, cap_chars=cc, cap_props=1024)
        assert rc == 0
        hdr, leaves, chars, props = emu_replay(batch, large=large)
        for d in range(batch.n_docs):
            diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
            assert not diffs, f"doc {d}: {diffs[:5]}"


@pytest.mark.parametrize("n_clients", [40, 63])
def test_many_writers_overflow_to_large_tier(orc, n_clients):
    """More than 31 writers (T3's 64 clients: the observer + 63): the small tier's 32-bit remove-client
    set overflows (FMT_E_CAPACITY, so the runtime escalates) and the large tier's W3 + W5 set holds
    them, with one prop set per writer's annotate value (up to 64 sets in W6); bit-exact vs the
    oracle."""
    batch = workloads.conflict_farm(8, n_clients=n_clients, ops_per_doc=1500, seed=13)
    assert batch.ops["client"].max() > 31
    small = emu_replay(batch)[0]
    assert (small["status"] == -3).any()
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=1024)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    assert (hdr["status"] == 0).all()
    assert any((leaves[d][: hdr[d]["n_leaves"]]["rm_clients"] >> np.uint64(32)).any() for d in range(batch.n_docs))
    assert hdr["n_props"].max() > 32
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


@pytest.mark.parametrize("n_clients", [8, 16, 24])
def test_inserts_with_props_match_oracle(orc, n_clients):
    """Insert ops whose segment spec carries props ({text, props}: TextSegment.make(text, props)):
    one- and two-key sets and an all-null set. Documents that overflow the small tier (more prop
    sets or writers than it holds) are compared from the large tier, as the runtime escalates them."""
    batch = workloads.with_insert_props(workloads.conflict_farm(30, n_clients=n_clients, ops_per_doc=1500, seed=19))
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    small = emu_replay(batch)
    large = emu_replay(batch, large=True)
    assert (large[0]["status"] == 0).all(), np.unique(large[0]["status"])
    assert set(np.unique(small[0]["status"])) <= {0, -3}
    for d in range(batch.n_docs):
        hdr, leaves, chars, props = small if int(small[0]["status"][d]) == 0 else large
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"


def test_large_tier_zamboni_matches_props_beyond_127_sets(orc):
    """Documents with hundreds of distinct prop sets (annotate values cycling over 400 texts): the
    large tier's zamboni compares prop-set ids of up to 1024 sets when it decides appends
    (matchProperties), not a 7-bit packing of them; bit-exact vs the oracle."""
    import copy

    batch = copy.copy(workloads.conflict_farm(6, n_clients=8, ops_per_doc=2000, seed=23))
    ann = np.nonzero(batch.ops["type"] == 2)[0]
    batch.ops = batch.ops.copy()
    batch.ops["payload"][ann] = np.arange(len(ann), dtype=np.uint32)
    batch.props_off = np.arange(len(ann) + 1, dtype=np.uint32)
    batch.props_kv = (1 + np.arange(len(ann), dtype=np.uint32) % 400)
    batch.values = ["null"] + [f'"v{i}"' for i in range(400)]
    batch.keys = ["k"]
    cl, cc, cp = emu_caps(large=True)
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=cp)
    assert rc == 0
    hdr, leaves, chars, props = emu_replay(batch, large=True)
    assert (hdr["status"] == 0).all() and hdr["n_props"].max() > 127
    for d in range(batch.n_docs):
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
