"""Reconnect churn: sequenced message streams in which every writer keeps reconnecting under a new
clientId (the production pattern behind the 63-writer cap).

`farm_messages` turns a generated conflict farm back into ISequencedDocumentMessage dicts (the
fmt_mt_op records, their inserted text and their annotate props). `churn` then renames a writer's
messages into a new session ("w3-17") at points where the writer has caught up: every earlier
message of that writer has seq <= the next message's refSeq. Across such a point the writer's
own unacked ops play no part in its perspective, so the renamed stream means exactly what the
original means, and every replay of it must reach the same state (client ids aside).
"""
import json
import random

from fluidframework_amd.streams import MT_ANNOTATE, MT_INSERT, MT_REMOVE, MergeTreeStreamBuilder


def _text(batch, off, n):
    return batch.text[off : off + n].tobytes().decode("utf-16-le", "surrogatepass")


def farm_messages(batch, d):
    """(initial text, [message dict]) of document d of a generated single-op-per-message farm."""
    o0, o1 = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
    init = ""
    if batch.doc_init is not None:
        off, n = (int(x) for x in batch.doc_init[d])
        init = _text(batch, off, n)
    msgs = []
    for r in batch.ops[o0:o1]:
        if int(r["flags"]) & 1:
            raise ValueError("GROUP messages are not expected in generated farms")
        t = int(r["type"])
        if t == MT_INSERT:
            op = {"pos1": int(r["pos1"]), "seg": _text(batch, int(r["payload"]), int(r["len"])), "type": t}
        elif t == MT_REMOVE:
            op = {"pos1": int(r["pos1"]), "pos2": int(r["pos2"]), "type": t}
        elif t == MT_ANNOTATE:
            pid = int(r["payload"])
            kv = batch.props_kv[int(batch.props_off[pid]) : int(batch.props_off[pid + 1])]
            props = {batch.keys[int(x) >> 16]: json.loads(batch.values[int(x) & 0xFFFF]) for x in kv}
            op = {"pos1": int(r["pos1"]), "pos2": int(r["pos2"]), "props": props, "type": t}
        else:
            raise ValueError(f"op type {t}")
        msgs.append({"clientId": f"w{int(r['client'])}", "sequenceNumber": int(r["seq"]),
                     "referenceSequenceNumber": int(r["ref_seq"]), "minimumSequenceNumber": int(r["min_seq"]),
                     "type": "op", "contents": op})
    return init, msgs


def churn(msgs, p=1.0, seed=0):
    """The same messages with writers renamed into sessions (a new one at a caught-up point with
    probability p). Returns (messages, number of distinct clientIds)."""
    rnd = random.Random(seed)
    last, session, out = {}, {}, []
    for m in msgs:
        w = m["clientId"]
        if w in last and last[w] <= m["referenceSequenceNumber"] and rnd.random() < p:
            session[w] = session.get(w, 0) + 1
        last[w] = m["sequenceNumber"]
        out.append(dict(m, clientId=f"{w}-{session.get(w, 0)}"))
    return out, len({m["clientId"] for m in out})


def session_writer(name):
    return name.rsplit("-", 1)[0] if "-" in name else name


def build(docs, remove_order=False, catchup=False):
    """docs: [(initial text, messages)] -> MergeTreeBatch through the stream builder."""
    b = MergeTreeStreamBuilder(keep_messages=True)
    for init, msgs in docs:
        d = b.begin_doc(init, observer="observer")
        for m in msgs:
            d.add_message(m)
    return b.finish(remove_order=remove_order, catchup=catchup)


def churned_farm(n_docs=4, ops_per_doc=3000, n_clients=8, p=1.0, seed=3, remove_order=False):
    """(original batch, churned batch, distinct clientIds per churned document)."""
    from fluidframework_amd import workloads

    src = workloads.conflict_farm(n_docs, n_clients=n_clients, ops_per_doc=ops_per_doc, seed=seed)
    orig, chd, counts = [], [], []
    for d in range(n_docs):
        init, msgs = farm_messages(src, d)
        cm, n = churn(msgs, p=p, seed=seed * 1000 + d)
        orig.append((init, msgs))
        chd.append((init, cm))
        counts.append(n)
    return build(orig, remove_order), build(chd, remove_order), counts
