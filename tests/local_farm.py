"""f4: streams of the LOCAL client — a Client whose own ops apply before they are
sequenced (client.ts:273-355), come back as acks (client.ts:1367-1368 → mergeTree.ts:1325-1408),
are rolled back (client.ts:554 → mergeTree.ts:2388-2514) or regenerated on reconnect
(client.ts:1452-1542). Each document of such a batch is one client's own view (the builder's
observer is that client).

Two sources:
- fixture_local_batch: the reference's conflict-farm replay fixtures (merge-tree/src/test/results,
  the messages of tests/golden/replay_msgs_0.40.json.gz) replayed from each WRITING client's
  perspective. The farm that recorded them (mergeTreeOperationRunner.ts:341-429) let every client
  create its ops of a round locally, on the state the previous rounds left, before any message of
  the round was sequenced; so a writer's stream is: its ops of the round as local submissions, then
  every message of the round (its own ones acknowledge them). The fixture's resultText after each
  round pins that client's text — reference-generated vectors for the local path.
- LocalFarm: generated farms (TestClient's role played by one oracle client per participant,
  test/testClient.ts), mirroring the conflict / reconnect / rollback farms
  (mergeTreeOperationRunner.ts:341-429, client.reconnectFarm.spec.ts:30-70,
  client.rollbackFarm.spec.ts:32-90): clients submit at their local view, the oldest sent op is
  sequenced and applied by everyone, newest unsent ops are rolled back, a client reconnects and
  regenerates its pending ops. Oracle-pinned (the reference itself cannot run here).
"""
from __future__ import annotations

import gzip
import json
import os
import random

import numpy as np

from fluidframework_amd.streams import (MT_ANNOTATE, MT_INSERT, MT_OP_DTYPE, MT_REMOVE,
                                        MergeTreeStreamBuilder, VALUE_ADJUST)

GOLDEN_MSGS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "replay_msgs_0.40.json.gz")


def load_fixture_msgs():
    return json.load(gzip.open(GOLDEN_MSGS, "rt", encoding="utf-8"))


def fixture_local_batch(stride=8, max_fixtures=None, clients=None):
    """One document per (fixture, writing client, checkpoint group): that client's local view of the
    stream up to the end of the group. Returns (batch, expected texts, [(fixture, client, group)])."""
    fixtures = load_fixture_msgs()[:max_fixtures]
    b = MergeTreeStreamBuilder()
    expected, where = [], []
    for fx in fixtures:
        groups = fx["groups"]
        writers = sorted({m["clientId"] for g in groups for m in g["msgs"]})
        for x in writers if clients is None else [c for c in writers if c in clients]:
            for k in range(0, len(groups), stride):
                d = b.begin_doc(initial_text=groups[0]["initialText"], observer=x)
                for g in range(k + 1):
                    start = groups[g]["msgs"][0]["sequenceNumber"] - 1 if groups[g]["msgs"] else None
                    for m in groups[g]["msgs"]:
                        if m["clientId"] == x:
                            assert m["referenceSequenceNumber"] == start  # made before the round's messages
                            d.local_op(m["contents"])
                    for m in groups[g]["msgs"]:
                        d.add_message(m)
                expected.append(groups[k]["resultText"])
                where.append((fx["name"], x, k))
    return b.finish(), expected, where


def fixture_local_docs(max_fixtures=None):
    """Every writing client's whole local stream of each 0.40 fixture (all 64 rounds) as its own
    single-document batch, with the fixture's final resultText: the `bench.py --workload local`
    sources (cycled to the bench's document count by workloads.replicate_batches)."""
    out = []
    for fx in load_fixture_msgs()[:max_fixtures]:
        groups = fx["groups"]
        for x in sorted({m["clientId"] for g in groups for m in g["msgs"]}):
            b = MergeTreeStreamBuilder()
            d = b.begin_doc(initial_text=groups[0]["initialText"], observer=x)
            for g in groups:
                for m in g["msgs"]:
                    if m["clientId"] == x:
                        d.local_op(m["contents"])
                for m in g["msgs"]:
                    d.add_message(m)
            out.append((f"{fx['name']}/{x}", b.finish(), groups[-1]["resultText"]))
    return out


class _Participant:
    def __init__(self, farm: "LocalFarm", name: str):
        from oracle import MergeTreeDoc  # (oracle/oracle.py: tests put oracle/ on sys.path)

        self.farm = farm
        self.name = name
        self.index = len(farm.b.docs)
        farm.log.append((self.index, "begin", farm.initial, name))
        self.doc = farm.b.begin_doc(initial_text=farm.initial, observer=name)
        self.orc = MergeTreeDoc()
        if farm.initial:
            self.orc.insert_local(0, farm.initial)
        self.orc.start_collab(0)
        self.applied = 0
        self.cur_seq = 0
        self.local_seq = 0
        self.by_local_seq: dict = {}  # localSeq -> the submitted op (regenerated ops keep theirs)
        self.pending: list = []       # [(localSeq, op, sent-message entry or None)] oldest first

    def sync(self):
        """Apply this client's recorded events to its oracle client."""
        if self.applied < len(self.doc.ops):
            recs = np.array(self.doc.ops[self.applied:], dtype=MT_OP_DTYPE)
            arena, poff, pkv = self.farm.tables()
            adj = self.farm.adjust_tables()
            if adj is not None:
                self.orc.set_adjusts(*adj)
            rel = self.farm.relpos_tables()
            if rel is not None:
                self.orc.set_relpos(*rel)
            self.orc.apply(recs, arena, poff, pkv)
            self.applied = len(self.doc.ops)

    def length(self) -> int:
        self.sync()
        return self.orc.local_length()


class LocalFarm:
    """A generated multi-client farm; every participant's own event stream is one document."""

    def __init__(self, seed, n_clients=4, initial="", min_length=8, keys=("a", "b", "c"), markers=True,
                 builder: MergeTreeStreamBuilder | None = None, new_ids=False, adjust=False, legacy=False):
        self.rnd = random.Random(seed)
        # legacy: a writer outside the farm ("R", an older client) whose sequenced inserts name their
        # position relative to a marker (relativePos1, client.ts:758-767 / mergeTree.ts:1462-1483)
        self.legacy = legacy
        self.legacy_ops = 0
        self.marker_ids: list[str] = []  # markerIds of the markers every participant has sequenced
        # adjust: half the annotates adjust the numeric key "w" (annotateAdjustRangeLocal, client.ts:286),
        # which raw annotates also set (numbers and a string, which an adjust reads as 0)
        self.adjust = adjust
        # new_ids: every reconnect comes back under a new clientId (as a real reconnect does); the
        # local client keeps its short id (startOrUpdateCollaboration, client.ts:1719-1725)
        self.new_ids = new_ids
        self.b = builder if builder is not None else MergeTreeStreamBuilder()
        self.initial = initial
        self.min_length = min_length
        self.keys = keys
        self.markers = markers
        self.seq = 0
        self.msn = 0
        self.inflight: list = []  # sent, not yet sequenced: [participant, op, ref, localSeq]
        # every builder call, (doc index, method, args...): replayable per document (replay_log)
        self.log: list = []
        self.parts = [_Participant(self, chr(ord("A") + i)) for i in range(n_clients)]
        self._arena_n = 0
        self._arena = np.zeros(0, dtype="<u2")
        self._props_n = -1
        self._props = None
        self.regens = 0
        self.rollbacks = 0

    # the builder's arena and props ops as the oracle reads them (batch-global value ids)
    def tables(self):
        if self._arena_n < len(self.b.text):
            self._arena = np.concatenate([self._arena] + self.b.text[self._arena_n:]).astype("<u2")
            self._arena_n = len(self.b.text)
        if self._props_n != len(self.b.props_list):
            off, kv = [0], []
            for t in self.b.props_list:
                for e in t:
                    kv += [(e[0] << 16) | e[1]] if len(e) == 2 else [(e[0] << 16) | VALUE_ADJUST, e[2]]
                off.append(len(kv))
            self._props = (np.asarray(off, dtype=np.uint32), np.asarray(kv, dtype=np.uint32))
            self._props_n = len(self.b.props_list)
        return self._arena, self._props[0], self._props[1]

    def relpos_tables(self):
        """(RELPOS_DTYPE table, "markerId" key id) of the builder so far, or None without any."""
        from fluidframework_amd.streams import MARKER_ID_KEY, NO_MARKER, RELPOS_DTYPE

        if not self.b.relpos and not self.legacy:
            return None
        # (a legacy farm from its first op: markers register under the markerId key as they arrive)
        key = (len(self.b.relpos), self.b.keys.ids.get(MARKER_ID_KEY, NO_MARKER))
        if getattr(self, "_rel_key", None) != key:
            self._rel = (np.array(self.b.relpos or [(NO_MARKER, 0, 0, 0)], dtype=RELPOS_DTYPE), key[1])
            self._rel_key = key
        return self._rel

    def legacy_op(self) -> bool:
        """R's relativePos1 insert next to a marker that every participant still holds unremoved
        (getMarkerFromId, mergeTree.ts:1450-1453: else the op names no marker), sequenced at once at
        the current seq (it reaches the service before anything in flight)."""
        from fluidframework_amd.streams import js_json

        r = self.rnd
        for _ in range(4):
            if not self.marker_ids:
                return False
            mid = r.choice(self.marker_ids)
            vid = self.b.values.ids.get(js_json(mid))
            if vid is None:
                return False
            ok = True
            for p in self.parts:
                p.sync()
                ok = ok and p.orc.marker_present(vid)
            if ok:
                break
        else:
            return False
        self.seq += 1
        msg = {"clientId": "R", "sequenceNumber": self.seq, "referenceSequenceNumber": self.seq - 1,
               "minimumSequenceNumber": self.msn, "type": "op",
               "contents": {"type": MT_INSERT, "relativePos1": {"id": mid, "before": r.random() < 0.5},
                            "seg": "rr"}}
        for q in self.parts:
            self.log.append((q.index, "add_message", msg))
            q.doc.add_message(msg)
            q.cur_seq = self.seq
        self.legacy_ops += 1
        return True

    def adjust_tables(self):
        """(ADJUST_DTYPE rows, value numbers) of the builder so far, or None without adjusts."""
        from fluidframework_amd.streams import ADJUST_DTYPE, value_numbers

        if not self.b.adjusts:
            return None
        key = (len(self.b.adjusts), len(self.b.values.items))
        if getattr(self, "_adj_key", None) != key:
            self._adj = (np.array(self.b.adjusts, dtype=ADJUST_DTYPE), value_numbers(self.b.values.items))
            self._adj_key = key
        return self._adj

    def _gen_op(self, p: _Participant):
        r = self.rnd
        n = p.length()
        if n == 0 or n < self.min_length or r.random() < 0.3:
            pos = r.randint(0, n)
            if self.markers and r.random() < 0.08:
                seg = {"marker": {"refType": 1}, "props": {"markerId": f"m{r.randrange(1 << 30)}"}}
            elif r.random() < 0.15:
                seg = {"text": p.name * r.randint(1, 3), "props": {r.choice(self.keys): r.randint(1, 4)}}
            else:
                seg = p.name * r.randint(1, 3)
            return {"type": MT_INSERT, "pos1": pos, "seg": seg}
        start = r.randint(0, n - 1)
        end = r.randint(start + 1, min(n, start + 1 + r.randint(1, 12)))
        if r.random() < 0.5:
            return {"type": MT_REMOVE, "pos1": start, "pos2": end}
        if self.adjust and r.random() < 0.5:
            a = {"delta": r.randint(-3, 3)}
            if r.random() < 0.3:
                a["min"] = r.randint(-4, 0)
            if r.random() < 0.3:
                a["max"] = r.randint(1, 6)
            return {"type": MT_ANNOTATE, "pos1": start, "pos2": end, "adjust": {"w": a}}
        if self.adjust and r.random() < 0.3:
            return {"type": MT_ANNOTATE, "pos1": start, "pos2": end, "props": {"w": r.choice([None, 0, 2, 5, "s"])}}
        props = {}
        for k in r.sample(self.keys, r.randint(1, len(self.keys))):
            props[k] = None if r.random() < 0.2 else r.choice([1, 2, 3, p.name, "x"])
        return {"type": MT_ANNOTATE, "pos1": start, "pos2": end, "props": props}

    def submit(self, p: _Participant):
        op = self._gen_op(p)
        self.log.append((p.index, "local_op", op))
        p.doc.local_op(op)
        p.local_seq += 1
        p.by_local_seq[p.local_seq] = op
        entry = [p, op, p.cur_seq, p.local_seq]
        p.pending.append((p.local_seq, op, entry))
        self.inflight.append(entry)

    def sequence_one(self):
        p, op, ref, _ = self.inflight.pop(0)
        self.seq += 1
        refs = [e[2] for e in self.inflight]
        msn = min(refs + [self.seq])
        self.msn = max(self.msn, min(msn, ref))
        msg = {"clientId": p.name, "sequenceNumber": self.seq, "referenceSequenceNumber": ref,
               "minimumSequenceNumber": self.msn, "type": "op", "contents": op}
        for q in self.parts:
            self.log.append((q.index, "add_message", msg))
            q.doc.add_message(msg)
            q.cur_seq = self.seq
        p.pending.pop(0)
        if op["type"] == MT_INSERT and isinstance(op.get("seg"), dict) and "marker" in op["seg"]:
            self.marker_ids.append(op["seg"]["props"]["markerId"])

    def rollback(self, p: _Participant) -> bool:
        """Roll back p's newest pending op if it is still unsent (the reference rolls back ops of a
        batch that never went out)."""
        if not p.pending:
            return False
        ls, op, entry = p.pending[-1]
        if entry is None or entry not in self.inflight or self.inflight[-1] is not entry:
            return False
        self.inflight.pop()
        p.pending.pop()
        self.log.append((p.index, "local_rollback"))
        p.doc.local_rollback()
        self.rollbacks += 1
        return True

    def reconnect(self, p: _Participant):
        """p's unsequenced ops are lost with its connection; regeneratePendingOp rebuilds them. As in
        the reference's reconnect farm (client.reconnectFarm.spec.ts:30-70), a client reconnects once
        every other client's sent op is sequenced: segment normalization (mergeTree.ts:2602-2612,
        "AB#34898: ... has some bugs") can order segments differently from remote clients when
        another client's older op is still in flight, which the reference's farms never exercise.
        So, as applyMessagesWithReconnect does, p's sent ops are dropped and every other client's
        is sequenced first."""
        self.inflight = [e for e in self.inflight if e[0] is not p]
        while self.inflight:
            self.sequence_one()
        if self.new_ids:
            p.name = f"{p.name.split('~')[0]}~{self.regens + 1}"
            self.log.append((p.index, "local_regen", None, p.name))
            p.doc.local_regen(None, p.name)
        else:
            self.log.append((p.index, "local_regen"))
            p.doc.local_regen()  # (the REGEN record; the pending ops follow once the oracle made them)
        p.sync()
        recs, text = p.orc.regen_take()
        new_ops = [self._regen_op(p, r, text) for r in recs]
        self.log.append((p.index, "regen_pending", new_ops))
        p.doc.regen_pending(new_ops)
        p.pending = []
        for r, op in zip(recs, new_ops):
            entry = [p, op, p.cur_seq, int(r["seq"])]
            p.pending.append((int(r["seq"]), op, entry))
            self.inflight.append(entry)
        self.regens += 1
        return recs, text

    @staticmethod
    def _regen_op(p: _Participant, r, text) -> dict:
        orig = p.by_local_seq[int(r["seq"])]
        t = int(r["type"])
        if t == MT_INSERT:
            n = int(r["len"]) | (int(r["flags"]) & 0x00FF0000)
            s = text[int(r["payload"]): int(r["payload"]) + n].tobytes().decode("utf-16-le", "surrogatepass")
            seg = orig["seg"]
            if isinstance(seg, dict) and "marker" in seg:
                new = seg
            elif isinstance(seg, dict):
                new = {"text": s, "props": seg.get("props")}
            else:
                new = s
            return {"type": MT_INSERT, "pos1": int(r["pos1"]), "seg": new}
        if t == MT_REMOVE:
            return {"type": MT_REMOVE, "pos1": int(r["pos1"]), "pos2": int(r["pos2"])}
        if "adjust" in orig:  # (regeneratePendingOp: an adjust op regenerates as one, client.ts:1186-1196)
            return {"type": MT_ANNOTATE, "pos1": int(r["pos1"]), "pos2": int(r["pos2"]), "adjust": orig["adjust"]}
        return {"type": MT_ANNOTATE, "pos1": int(r["pos1"]), "pos2": int(r["pos2"]), "props": orig["props"]}

    def run(self, steps, p_submit=0.45, p_rollback=0.08, p_reconnect=0.03, drain=True):
        r = self.rnd
        writers = self.parts[1:]  # client A only reads (the farms' baseline client)
        for _ in range(steps):
            x = r.random()
            if x < p_submit or not self.inflight:
                self.submit(r.choice(writers))
            elif x < p_submit + p_rollback:
                self.rollback(r.choice(writers))
            elif x < p_submit + p_rollback + p_reconnect:
                self.reconnect(r.choice(writers))
            elif self.legacy and x < p_submit + p_rollback + p_reconnect + 0.1:
                self.legacy_op()
            else:
                self.sequence_one()
        if drain:
            while self.inflight:
                self.sequence_one()
        return self

    def texts(self):
        out = []
        for p in self.parts:
            p.sync()
            out.append(p.orc.text())
        return out


def farm_log(farms) -> list:
    """The builder calls of the farms, document by document (each document's own calls in order):
    what a packer that writes documents contiguously (js/fmt.js) replays."""
    log = [e for f in farms for e in f.log]
    return sorted(log, key=lambda e: e[0])  # (stable: each document keeps its order)


def replay_log(log, builder=None) -> MergeTreeStreamBuilder:
    """The calls of farm_log on a (fresh) Python builder."""
    b = builder if builder is not None else MergeTreeStreamBuilder()
    docs = {}
    for e in log:
        if e[1] == "begin":
            docs[e[0]] = b.begin_doc(initial_text=e[2], observer=e[3])
        else:
            getattr(docs[e[0]], e[1])(*e[2:])
    return b


def local_farm_batch(seeds, steps=300, **kw):
    """Several farms in one batch (every participant's view is a document). Returns (batch, farms)."""
    b = MergeTreeStreamBuilder()
    farms = [LocalFarm(sd, builder=b, **kw).run(steps) for sd in seeds]
    return b.finish(), farms
