"""Annotate-adjust (SURVEY §8 a10's IEEE-double half): IMergeTreeAnnotateAdjustMsg.adjust
(merge-tree/src/ops.ts:187-222) folded by computePropertyValue (segmentPropertiesManager.ts:54-78).

The reference's fixtures hold no adjust op, so parity is anchored three ways:
  - hand cases whose expected values are worked out from computePropertyValue's text (number or 0,
    + delta, max checked before min, a null min/max compared as 0 and assigned, -0 === 0, float sums);
  - the reference's conflict-farm fixtures (replay_msgs_0.40) with their annotates rewritten into
    adjusts and raw numbers on the same keys: the final texts still equal the fixtures' resultText,
    and the emulated engine (small tier, and the large tier the runtime escalates to) equals the
    oracle restatement bit for bit, computed-number tables included;
  - legacy summaries read getAtSeq(minSeq), which the oracle restates with each segment's
    PropertiesManager (msnConsensus + pending remote changes, updateMsn at handleProperties and at
    zamboni's peek, copyTo on splits) and the engine keeps as per-leaf records: the Python host over
    the engine's legacy prop sets equals the oracle's SnapshotLegacy restatement byte for byte.
"""
import gzip
import json
import os
import random

import numpy as np
import pytest

from fluidframework_amd import summary
from fluidframework_amd.streams import VALUE_COMPUTED, MergeTreeStreamBuilder, UnsupportedOp, js_number
from mt_compare import compare_doc, emu_caps, emu_legacy_props, emu_numbers, emu_replay, visible_text

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "replay_msgs_0.40.json.gz")


def _msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "contents": contents}


def _ann(p1, p2, props=None, adjust=None):
    op = {"type": 2, "pos1": p1, "pos2": p2}
    if props is not None:
        op["props"] = props
    if adjust is not None:
        op["adjust"] = adjust
    return op


def hand_cases():
    """(initial text, messages, expected value of key per character: list of dicts)."""
    cases = []
    # absent key → 0 + delta; raw number + delta; a string value counts as 0
    cases.append(("abc", [_msg("B", 1, 0, _ann(0, 1, props={"n": 5})), _msg("B", 2, 1, _ann(1, 2, props={"n": "x"})),
                          _msg("C", 3, 0, _ann(0, 3, adjust={"n": {"delta": 2}}))],
                  [{"n": 7}, {"n": 2}, {"n": 2}]))
    # max is checked before min (min > max: the max wins); min clamps below
    cases.append(("ab", [_msg("B", 1, 0, _ann(0, 1, adjust={"n": {"delta": 7, "min": 10, "max": 5}})),
                         _msg("B", 2, 1, _ann(1, 2, adjust={"n": {"delta": -3, "min": -1}}))],
                  [{"n": 5}, {"n": -1}]))
    # a null max: `adjusted > null` compares with 0 and assigns null, which deletes the key; a null
    # min likewise when the sum is negative; a null delta adds 0
    cases.append(("abc", [_msg("B", 1, 0, _ann(0, 3, props={"n": 1, "k": 1})),
                          _msg("B", 2, 1, _ann(0, 1, adjust={"n": {"delta": 1, "max": None}})),
                          _msg("B", 3, 2, _ann(1, 2, adjust={"n": {"delta": -5, "min": None}})),
                          _msg("B", 4, 3, _ann(2, 3, adjust={"n": {"delta": None}}))],
                  [{"k": 1}, {"k": 1}, {"n": 1, "k": 1}]))
    # floats: the sum is IEEE double (0.1 + 0.2), JSON.stringify forms (1e-7, 0.00001)
    cases.append(("abcd", [_msg("B", 1, 0, _ann(0, 4, adjust={"n": {"delta": 0.1}})),
                           _msg("C", 2, 1, _ann(0, 1, adjust={"n": {"delta": 0.2}})),
                           _msg("C", 3, 2, _ann(1, 2, adjust={"n": {"delta": -0.0999999}})),
                           _msg("C", 4, 3, _ann(2, 3, adjust={"n": {"delta": -0.09999}}))],
                  [{"n": 0.1 + 0.2}, {"n": 0.1 - 0.0999999}, {"n": 0.1 - 0.09999}, {"n": 0.1}]))
    # raw then adjust of one key in one op (opToChanges: props entries first); -0 behaves as 0
    cases.append(("ab", [_msg("B", 1, 0, _ann(0, 2, props={"n": 3}, adjust={"n": {"delta": 1}})),
                         _msg("B", 2, 1, _ann(1, 2, props={"n": -0.0}, adjust={"n": {"delta": -0.0}}))],
                  [{"n": 4}, {"n": 0}]))
    # a computed number equal to a host value takes the host's id (=== matching for zamboni/summary)
    cases.append(("ab", [_msg("B", 1, 0, _ann(0, 1, props={"n": 6})), _msg("B", 2, 1, _ann(1, 2, props={"n": 4})),
                         _msg("C", 3, 2, _ann(1, 2, adjust={"n": {"delta": 2}}))],
                  [{"n": 6}, {"n": 6}]))
    return cases


def _batch(cases):
    b = MergeTreeStreamBuilder()
    for init, msgs, _ in cases:
        d = b.begin_doc(init)
        for m in msgs:
            d.add_message(m)
    return b.finish()


def _char_props(hdr, leaves, chars, props, batch, numbers):
    vals = summary.values_with_numbers(batch.values, numbers)
    out = []
    for L in leaves[: int(hdr["n_leaves"])]:
        if int(L["rm_seq"]) != 0x7FFFFFFF:
            continue
        pid = int(L["props"])
        kv = [] if pid == 0xFFFF else [int(x) for x in props[pid]["kv"][: props[pid]["n"]]]
        d = {batch.keys[x >> 16]: json.loads(vals[x & 0xFFFF]) for x in kv}
        out += [d] * int(L["len"])
    return out


def test_packer_writes_adjust_rows():
    batch = _batch(hand_cases())
    assert batch.adjusts is not None and batch.value_num is not None
    assert len(batch.value_num) == len(batch.values)
    i = batch.values.index("5")
    assert batch.value_num[i] == 5.0 and np.isnan(batch.value_num[batch.values.index('"x"')])
    assert np.isnan(batch.value_num[0])  # "null"


def test_oracle_hand_cases(orc):
    cases = hand_cases()
    batch = _batch(cases)
    nums = []
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=64, cap_chars=64, cap_props=64, numbers=nums)
    assert rc == 0
    for d, (_, _, want) in enumerate(cases):
        got = _char_props(oh[d], ol[d], oc[d], op[d], batch, nums[d])
        assert got == want, (d, got, want)
    # host ids serve computed numbers equal to a host value ("6" of case 5, "5" of case 1, a batch-wide
    # dictionary): those documents compute only what no host text holds
    assert len(nums[5]) == 0 and list(nums[1]) == [-1.0]


def test_engine_hand_cases(orc):
    batch = _batch(hand_cases())
    nums = []
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, cap_leaves=512, cap_chars=6144, cap_props=1024, numbers=nums)
    hdr, leaves, chars, props = emu_replay(batch)
    for d in range(batch.n_docs):
        assert not compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d])), d
        assert np.array_equal(emu_numbers(d), nums[d]), d


def adjust_fixture_batch(exact_tail=False, seed=11, narrow=False, messages=False):
    """The reference's conflict-farm fixtures with every annotate rewritten: adjusts of "n" (and "w")
    with deltas from {1, -2, 0.5, 0.1, -0.3, 1e-7 …} and sometimes min/max clamps (null ones too), raw
    numbers on "n", nulls, or the original {"client"} props. With exact_tail, annotates above the
    document's final minSeq keep their original props (another key), so its legacy summary is exact.
    With narrow, deltas are ±1 / 2 clamped to [0, 4] (few distinct values: documents fit the small
    tier's 32 prop sets). With messages, returns [(initial text, messages, final text)] instead."""
    fx = json.load(gzip.open(GOLDEN, "rt", encoding="utf-8"))
    rng = random.Random(seed)
    deltas = [1, -2, 0.5, 0.1, -0.3, 3, 1e-7, -0.25, 7]

    def rewrite(op):
        if op.get("type") != 2:
            return op
        r = rng.random()
        if narrow:
            op = {k: v for k, v in op.items() if k != "props"}
            if r < 0.2:
                op["props"] = {"n": rng.choice([1, 3])}
            else:
                op["adjust"] = {"n": {"delta": rng.choice([1, -1, 2]), "min": 0, "max": 4}}
            return op
        op = {k: v for k, v in op.items() if k != "props"}
        if r < 0.15:
            op["props"] = {"n": rng.choice([1, 2, 5, 0.5, "s"])}
        elif r < 0.2:
            op["props"] = {"n": None}
        elif r < 0.3:
            op["props"] = {"client": "X"}
        else:
            a = {"delta": rng.choice(deltas)}
            if rng.random() < 0.3:
                a["max"] = rng.choice([4, 10, 2.5, None])
            if rng.random() < 0.3:
                a["min"] = rng.choice([-3, 0, -0.5, None])
            op["adjust"] = {"n": a}
            if rng.random() < 0.2:
                op["adjust"]["w"] = {"delta": rng.choice(deltas)}
            if rng.random() < 0.1:
                op["props"] = {"n": 2}
        return op

    docs = []
    for f in fx:
        g = f["groups"]
        msgs = [m for gg in g for m in gg["msgs"]]
        final_msn = msgs[-1]["minimumSequenceNumber"]
        out = []
        for m in msgs:
            c = m["contents"]
            if not (exact_tail and m["sequenceNumber"] > final_msn):
                if c.get("type") == 3:
                    c = dict(c, ops=[rewrite(o) for o in c["ops"]])
                else:
                    c = rewrite(c)
            out.append(dict(m, contents=c))
        docs.append((g[0]["initialText"], out, g[-1]["resultText"]))
    if messages:
        return docs
    b = MergeTreeStreamBuilder(keep_messages=True)
    for init, msgs, _ in docs:
        d = b.begin_doc(init, observer="A")
        for m in msgs:
            d.add_message(m)
    return b.finish(), [f for _, _, f in docs]


@pytest.mark.parametrize("exact_tail", [False, True])
def test_oracle_adjust_farms_keep_fixture_texts(orc, exact_tail):
    batch, finals = adjust_fixture_batch(exact_tail)
    assert batch.adjusts is not None and len(batch.adjusts) > 10
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=4096, cap_chars=1 << 16, cap_props=1024)
    assert rc == 0
    for d in range(batch.n_docs):
        assert visible_text(oh[d], ol[d], oc[d]) == finals[d], d


@pytest.mark.parametrize("large", [False, True])
def test_engine_adjust_farms_match_oracle(orc, large):
    batch, finals = adjust_fixture_batch(narrow=not large)
    cl, cc, cp = emu_caps(large)
    nums = []
    rc, oh, ol, oc, op, _ = orc.mt_replay_batch(batch, threads=8, cap_leaves=cl, cap_chars=cc, cap_props=cp,
                                                numbers=nums)
    hdr, leaves, chars, props = emu_replay(batch, large=4 if large else False)
    computed = 0
    for d in range(batch.n_docs):
        if not large and oh[d]["status"] == 0 and hdr[d]["status"] == -3:
            continue  # outgrew the small tier: the runtime replays it in the large tier
        assert hdr[d]["status"] == oh[d]["status"], d
        diffs = compare_doc((oh[d], ol[d], oc[d], op[d]), (hdr[d], leaves[d], chars[d], props[d]))
        assert not diffs, f"doc {d}: {diffs[:5]}"
        assert np.array_equal(emu_numbers(d), nums[d]), d
        assert visible_text(hdr[d], leaves[d], chars[d]) == finals[d]
        computed += len(nums[d]) + 1
    assert computed > (50 if large else 3)


def test_legacy_summaries_match_oracle(orc):
    """getAtSeq(minSeq) (segmentPropertiesManager.ts:328-344, via snapshotlegacy.ts:211-212): every
    adjusted document's legacy summary from the engine's per-leaf legacy prop sets (the emulated
    PropertiesManager records) equals the oracle's SnapshotLegacy restatement over its own managers,
    with adjusts above the final minSeq (the common case) and without."""
    differs = 0
    for exact_tail in (True, False):
        batch, _ = adjust_fixture_batch(exact_tail)
        hdr, leaves, chars, props = emu_replay(batch, large=4)
        for d in range(batch.n_docs):
            h = hdr[d]
            assert int(h["status"]) == 0, d
            vals = summary.values_with_numbers(batch.values, emu_numbers(d))
            legacy = emu_legacy_props(d)
            assert legacy is not None
            got = summary.legacy_summary(h, leaves[d], chars[d], props[d], batch.keys, vals, legacy_props=legacy)
            want = orc.mt_replay_summary(batch, d, batch.keys, batch.values)
            assert got == want, d
            now = summary.legacy_summary(h, leaves[d], chars[d], props[d], batch.keys, vals)
            differs += now != got
    assert differs > 0  # pending changes above minSeq make getAtSeq differ from the current properties


def test_legacy_summaries_match_oracle_small_tier(orc):
    """The same through the small tier alone (narrow deltas: documents fit its 32 prop sets), and with
    the legacy prop sets the getAtSeq evaluation interns at the end of the replay."""
    batch, _ = adjust_fixture_batch(narrow=True)
    hdr, leaves, chars, props = emu_replay(batch)
    checked = 0
    for d in range(batch.n_docs):
        h = hdr[d]
        if int(h["status"]) != 0:
            continue  # (outgrew the small tier: the large tier replays it)
        vals = summary.values_with_numbers(batch.values, emu_numbers(d))
        got = summary.legacy_summary(h, leaves[d], chars[d], props[d], batch.keys, vals, legacy_props=emu_legacy_props(d))
        assert got == orc.mt_replay_summary(batch, d, batch.keys, batch.values), d
        checked += 1
    assert checked > 3


def getatseq_cases():
    """(initial text, messages, expected legacy segmentTexts) worked out by hand from
    segmentPropertiesManager.ts (handleProperties :188-238, updateMsn :275-291, getAtSeq :328-344) and
    zamboni.ts:44 (updateMsn on the peeked segment when minSeq advances)."""
    ins = lambda p, t: {"type": 0, "pos1": p, "seg": t}  # noqa: E731
    return [
        # a raw change that arrives while an adjust is pending is queued: at minSeq 1 the adjust's
        # result shows, not the later raw value
        ("ab", [_msg("B", 1, 0, _ann(0, 2, adjust={"n": {"delta": 1}})), _msg("B", 2, 1, _ann(0, 2, props={"n": 5})),
                _msg("C", 3, 2, ins(2, "x"), msn=1)],
         [{"text": "ab", "props": {"n": 1}}]),
        # the adjust was folded (zamboni's updateMsn when minSeq reached it) before the raw change came:
        # the raw change folds straight into msnConsensus, so it shows although its seq is above minSeq
        ("ab", [_msg("B", 1, 0, _ann(0, 2, adjust={"n": {"delta": 1}})), _msg("C", 2, 1, ins(2, "x"), msn=1),
                _msg("B", 3, 2, _ann(0, 2, props={"n": 5}), msn=1)],
         [{"text": "ab", "props": {"n": 5}}]),
        # a key deleted now (null queued behind an adjust) but alive at minSeq goes last
        ("ab", [_msg("B", 1, 0, _ann(0, 2, props={"n": 2, "a": 1})), _msg("B", 2, 1, _ann(0, 2, adjust={"n": {"delta": 1}})),
                _msg("B", 3, 2, _ann(0, 2, props={"n": None})), _msg("C", 4, 3, ins(2, "x"), msn=2)],
         [{"text": "ab", "props": {"a": 1, "n": 3}}]),
        # a split copies the manager (copyTo): both halves keep the pending adjust
        ("abcd", [_msg("B", 1, 0, _ann(0, 4, adjust={"n": {"delta": 2}})), _msg("B", 2, 1, _ann(2, 4, props={"n": 9})),
                  _msg("C", 3, 2, ins(4, "x"), msn=1)],
         [{"text": "abcd", "props": {"n": 2}}]),
    ]


def test_getatseq_hand_cases(orc):
    cases = getatseq_cases()
    b = MergeTreeStreamBuilder()
    for init, msgs, _ in cases:
        d = b.begin_doc(init, observer="A")
        for m in msgs:
            d.add_message(m)
    batch = b.finish()
    hdr, leaves, chars, props = emu_replay(batch)
    for d, (_, _, want) in enumerate(cases):
        head, body = orc.mt_replay_summary(batch, d, batch.keys, batch.values)
        assert body is None and json.loads(head)["segmentTexts"] == want, (d, head)
        vals = summary.values_with_numbers(batch.values, emu_numbers(d))
        got = summary.legacy_summary(hdr[d], leaves[d], chars[d], props[d], batch.keys, vals, legacy_props=emu_legacy_props(d))
        assert got == (head, body), d
        assert json.loads(got[0])["segmentTexts"] == want  # (JSON key order too: json.loads keeps it)
        assert list(json.loads(got[0])["segmentTexts"][0]["props"]) == list(want[0]["props"])


def test_computed_numbers_format_like_json_stringify():
    assert summary.values_with_numbers(["null"], [0.1 + 0.2, 1e-7, 1e21])[VALUE_COMPUTED:] == [
        "0.30000000000000004", "1e-7", "1e+21"]
    assert js_number(-0.0) == "0"
