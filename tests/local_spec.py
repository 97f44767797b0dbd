"""Runs the reference's local-client spec cases transcribed as data (tests/golden/local_spec_cases.json:
client.rollback.spec.ts, client.applyMsg.spec.ts, resetPendingSegmentsToOp.spec.ts).

A case names its clients; each client's own event stream (its local submissions, the messages it
applies, its rollbacks and reconnects) is one document whose observer is that client. Reconnects
need the regenerated ops to make the resubmitted messages: the interpreter keeps one interactive
oracle client per participant (tests/local_farm.py _Participant, test infrastructure), as the
reference's TestClient would regenerate them. Every check becomes a checkpoint document (the
client's events up to that step), replayed by a runner — the oracle's batch replay, the emulated
engine or libfmt.so — and its expectations are evaluated on that runner's converged state.
"""
from __future__ import annotations

import json
import os

import numpy as np

from fluidframework_amd.streams import (LOCAL_SEQ_BASE, MT_ANNOTATE, MT_GROUP, MT_INSERT, MT_OP_DTYPE, MT_REMOVE,
                                        MergeTreeStreamBuilder)
from local_farm import LocalFarm, _Participant
from mt_compare import resolve_props, visible_text

CASES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "local_spec_cases.json")
NOT_REMOVED = 0x7FFFFFFF


def load_cases():
    with open(CASES, encoding="utf-8") as f:
        return json.load(f)["cases"]


class SpecRun:
    def __init__(self, case: dict):
        self.case = case
        self.farm = LocalFarm(0, n_clients=0, initial=case.get("initial", ""))
        self.parts = {c: _Participant(self.farm, c) for c in case["clients"]}
        self.msgs: dict = {}
        self.tags: dict = {}
        self.checks: list = []  # (client, number of its events, expectations, step index)
        for k, step in enumerate(case["steps"]):
            getattr(self, "_" + step[0])(*step[1:]) if step[0] != "check" else self._check(k, *step[1:])

    # ---- events (each recorded in farm.log, as the farms do)
    def _ev(self, p: _Participant, method: str, *args):
        self.farm.log.append((p.index, method) + args)
        getattr(p.doc, method)(*args)

    def _local(self, c, op, tag=None):
        p = self.parts[c]
        self._ev(p, "local_op", op)
        p.local_seq += 1
        p.by_local_seq[p.local_seq] = op
        if tag is not None:
            self.tags[tag] = op

    def _message(self, c, op, seq, opts=None):
        opts = opts or {}
        p = self.parts[c]
        self.msgs[seq] = {"clientId": opts.get("clientId", c), "sequenceNumber": seq,
                          "referenceSequenceNumber": opts.get("ref", p.cur_seq),
                          "minimumSequenceNumber": opts.get("msn", 0), "type": "op", "contents": op}

    def _send(self, c, op_or_tag, seq, opts=None):
        if isinstance(op_or_tag, str):
            op = self.tags[op_or_tag]
        else:
            op = op_or_tag
            self._local(c, op)
        self._message(c, op, seq, opts)

    def _apply(self, seq, clients):
        for c in self.case["clients"] if clients == "all" else clients:
            p = self.parts[c]
            self._ev(p, "add_message", self.msgs[seq])
            p.cur_seq = seq

    def _rollback(self, c):
        self._ev(self.parts[c], "local_rollback")

    def _regen(self, c, seqs, opts=None):
        p = self.parts[c]
        self._ev(p, "local_regen")
        p.sync()
        recs, text = p.orc.regen_take()
        new_ops = [LocalFarm._regen_op(p, r, text) for r in recs]
        self._ev(p, "regen_pending", new_ops)
        groups: list = []  # one resubmitted message per original op (localSeq), in order
        for r, op in zip(recs, new_ops):
            if groups and groups[-1][0] == int(r["seq"]):
                groups[-1][1].append(op)
            else:
                groups.append((int(r["seq"]), [op]))
        assert len(seqs) in (0, len(groups)), (seqs, len(groups))
        for seq, (_, ops) in zip(seqs, groups):
            self._message(c, ops[0] if len(ops) == 1 else {"type": MT_GROUP, "ops": ops}, seq, opts)

    def _check(self, k, who, expect):
        names = self.case["clients"] if who == "all" else [who] if isinstance(who, str) else who
        for c in names:
            p = self.parts[c]
            if "pending" in expect:  # (the interactive oracle client: pendingSegments.length)
                p.sync()
                assert p.orc.pending_groups() == expect["pending"], \
                    f"{self.case['name']} step {k} client {c}: pending {p.orc.pending_groups()} != {expect['pending']}"
            n = sum(1 for e in self.farm.log if e[0] == p.index)
            self.checks.append((c, n, expect, k))

    # ---- macros
    def _ins_chars(self, c, text):
        for i, ch in enumerate(text):
            self._local(c, {"type": MT_INSERT, "pos1": self.parts[c].length(), "seg": ch})

    def _ins_ack_each(self, c, text):
        p = self.parts[c]
        for ch in text:
            op = {"type": MT_INSERT, "pos1": p.length(), "seg": ch}
            self._local(c, op)
            cur = p.cur_seq
            self._message(c, op, cur + 1, {"ref": cur, "msn": cur})
            self._apply(cur + 1, [c])

    def _ins_nested(self, c, n, text):
        for i in range(n):
            self._local(c, {"type": MT_INSERT, "pos1": i, "seg": text}, f"n{i}")

    def _applymsg_interleaved(self, c, n):
        """client.applyMsg.spec.ts:48-83, positions from the local length at each step."""
        p = self.parts[c]
        for i in range(n):
            ln = p.length()
            pos1 = ln // 2
            m = i % 6
            if m in (0, 5):
                op = {"type": MT_REMOVE, "pos1": pos1, "pos2": max((ln - pos1) // 4 - m + pos1, pos1 + 1)}
            elif m in (1, 4):
                op = {"type": MT_INSERT, "pos1": pos1, "seg": str(i) * (m + 5)}
            else:
                op = {"type": MT_ANNOTATE, "pos1": pos1, "pos2": max((ln - pos1) // 3 - m + pos1, pos1 + 1),
                      "props": {"foo": str(i)}}
            self._send(c, op, i + 1)
        for i in range(n):
            self._apply(i + 1, [c])

    # ---- checkpoint documents
    def checkpoint_batch(self, builder: MergeTreeStreamBuilder | None = None):
        """One document per (check, client): that client's events up to the check. Returns the
        builder and the [(case, client, expectations, step)] of its documents (appended in order)."""
        b = builder if builder is not None else MergeTreeStreamBuilder()
        where = []
        for c, n, expect, k in self.checks:
            p = self.parts[c]
            events = [e for e in self.farm.log if e[0] == p.index][:n]
            d = None
            for e in events:
                if e[1] == "begin":
                    d = b.begin_doc(initial_text=e[2], observer=e[3])
                else:
                    getattr(d, e[1])(*e[2:])
            where.append((self.case["name"], c, expect, k))
        return b, where


VALUE_COMPUTED = 0x8000  # fmt.h FMT_MT_VALUE_COMPUTED: annotate-adjust results, the document's numbers


def _value(batch, v, numbers):
    if v >= VALUE_COMPUTED:
        x = float(numbers[v - VALUE_COMPUTED])
        return int(x) if x.is_integer() else x
    return json.loads(batch.values[v])


def _props_dict(batch, table, pid, numbers=()):
    kv = resolve_props(int(pid), table)
    if kv is None:
        return {}
    return {batch.keys[e >> 16]: _value(batch, e & 0xFFFF, numbers) for e in kv}


def _local_view(leaves):
    """(leaf, start position) of every leaf in the local view (not removed)."""
    out, pos = [], 0
    for L in leaves:
        if int(L["rm_seq"]) == NOT_REMOVED:
            out.append((L, pos))
            pos += int(L["len"])
    return out


def _props_at(batch, leaves, table, pos, numbers=()):
    for L, s in _local_view(leaves):
        if s <= pos < s + int(L["len"]):
            return _props_dict(batch, table, L["props"], numbers)
    raise AssertionError(f"position {pos} outside the local view")


def _stamp(v):
    return LOCAL_SEQ_BASE | int(v.split(":")[1]) if isinstance(v, str) else int(v)


def _regen_insert_props(batch, ops, k):
    op = ops[k]
    assert int(op["type"]) == MT_INSERT, f"regenerated op {k} is not an insert"
    pos2 = int(op["pos2"])
    if pos2 <= 0:
        return None
    return {batch.keys[e >> 16]: (None if (e & 0xFFFF) == 0 else json.loads(batch.values[e & 0xFFFF]))
            for e in batch.props_kv[batch.props_off[pos2 - 1]: batch.props_off[pos2 - 1 + 1]]}


def evaluate(batch, where, results, regen_of, numbers_of=None):
    """results[d] = (header, leaves[:n], chars, props table) of checkpoint document d; regen_of(d) =
    (ops, text); numbers_of(d) = its computed annotate-adjust numbers (adjust batches). Returns a list
    of failures."""
    fails = []
    texts: dict = {}
    for d, (name, c, expect, k) in enumerate(where):
        h, leaves, chars, props = results[d]
        tag = f"{name} / step {k} / client {c}"
        if "status" in expect:
            if int(h["status"]) != expect["status"]:
                fails.append(f"{tag}: status {int(h['status'])} != {expect['status']}")
            continue
        if int(h["status"]) != 0:
            fails.append(f"{tag}: status {int(h['status'])}")
            continue
        text = visible_text(h, leaves, chars)
        texts.setdefault((name, k), []).append(text)
        for key, v in expect.items():
            if key == "text" and text != v:
                fails.append(f"{tag}: text {text!r} != {v!r}")
            elif key == "markers":
                n = sum(1 for L, _ in _local_view(leaves) if int(L["pad"]) & 0x8000)
                if n != v:
                    fails.append(f"{tag}: {n} markers != {v}")
            elif key in ("props", "props_range"):
                items = ([(int(p), p, e) for p, e in v.items()] if key == "props"
                         else [(i, i, e) for s, t, e in v for i in range(s, t)])
                nums = numbers_of(d) if numbers_of is not None else ()
                for pos, _, e in items:
                    got = _props_at(batch, leaves, props, pos, nums)
                    for pk, pv in e.items():
                        if got.get(pk) != pv:
                            fails.append(f"{tag}: props at {pos}: {pk}={got.get(pk)!r} != {pv!r}")
            elif key == "leaf":
                for i, e in v:
                    for f, want in e.items():
                        if int(leaves[i][f]) != _stamp(want):
                            fails.append(f"{tag}: leaf {i} {f} {int(leaves[i][f])} != {_stamp(want)}")
            elif key == "all_acked":
                bad = [int(L["ins_seq"]) for L in leaves if LOCAL_SEQ_BASE <= int(L["ins_seq"]) < NOT_REMOVED] + \
                      [int(L["rm_seq"]) for L in leaves if LOCAL_SEQ_BASE <= int(L["rm_seq"]) < NOT_REMOVED]
                if bad:
                    fails.append(f"{tag}: pending stamps left {bad[:4]}")
            elif key == "no_rolled_back":
                if any(int(L["ins_seq"]) == -2 for L in leaves):
                    fails.append(f"{tag}: a rolled-back leaf is still linked")
            elif key == "min_seq" and int(h["min_seq"]) != v:
                fails.append(f"{tag}: min_seq {int(h['min_seq'])} != {v}")
            elif key == "regen_count":
                n = len(regen_of(d)[0])
                if n != v:
                    fails.append(f"{tag}: {n} regenerated ops != {v}")
            elif key == "regen_insert_props":
                ops = regen_of(d)[0]
                for i, want in v:
                    got = _regen_insert_props(batch, ops, i)
                    if got != want:
                        fails.append(f"{tag}: regenerated insert {i} props {got} != {want}")
    for d, (name, c, expect, k) in enumerate(where):
        if expect.get("same_text") and len(set(texts.get((name, k), []))) > 1:
            fails.append(f"{name} / step {k}: clients differ {texts[(name, k)]}")
    return fails


def spec_batch(cases=None, adjust=False):
    """Every case's checkpoint documents in one batch: (batch, where). adjust: the annotate-adjust
    cases ("adjust": true), which run as a batch of their own, instead of the others."""
    b = MergeTreeStreamBuilder()
    where = []
    for case in load_cases() if cases is None else cases:
        if bool(case.get("adjust")) != adjust:
            continue
        _, w = SpecRun(case).checkpoint_batch(b)
        where += w
    return b.finish(), where
