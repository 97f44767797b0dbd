"""Generated marker-rich SharedString message streams (tests only): every document inserts Markers
with its own markerId values, annotates ranges, and inserts at positions relative to its markers —
the shape that gives a batch of many documents more distinct property values than 16-bit
batch-global ids hold (fmt.h doc_value_base)."""
import random

from fluidframework_amd.streams import MergeTreeStreamBuilder


def _msg(client, seq, ref, contents, msn):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "contents": contents}


def doc_messages(d: int, n_ops: int, seed: int, adjust: bool = False, wide: int = 0):
    """(initial text, messages) of document d: one writer per message, refSeq = seq - 1, minSeq
    trailing by up to 8, so every position is in the op's own view."""
    rnd = random.Random(seed * 1_000_003 + d)
    init = "the quick brown fox"
    length, markers, msgs, msn = len(init), [], [], 0
    for seq in range(1, n_ops + 1):
        client = "AB"[seq % 2]
        msn = max(msn, seq - 1 - rnd.randint(0, 8))
        kind = rnd.random()
        if kind < 0.3:
            mid = f"d{d}-m{seq}"
            op = {"type": 0, "pos1": rnd.randint(0, length),
                  "seg": {"marker": {"refType": 1}, "props": {"markerId": mid, "label": f"L{seq % 7}"}}}
            markers.append(mid)
            length += 1
        elif kind < 0.5 and markers:
            op = {"type": 0, "relativePos1": {"id": rnd.choice(markers), "before": rnd.random() < 0.5}, "seg": "rel"}
            length += 3
        elif kind < 0.7 and length > 2:
            p = rnd.randint(0, length - 2)
            if adjust and rnd.random() < 0.5:
                op = {"type": 2, "pos1": p, "pos2": p + 2, "adjust": {"weight": {"delta": rnd.randint(-3, 3)}}}
            elif wide:  # a formatting run: `wide` keys at once, some of them deleted (null)
                keys = rnd.sample(range(wide + 6), wide)
                op = {"type": 2, "pos1": p, "pos2": p + 2,
                      "props": {f"k{k}": (None if rnd.random() < 0.1 else rnd.randint(0, 3)) for k in keys}}
            else:
                op = {"type": 2, "pos1": p, "pos2": p + 2, "props": {"color": f"c{d}-{rnd.randint(0, 40)}",
                                                                    "n": rnd.randint(0, 5000)}}
        else:  # (no removes: a relative position must find its marker)
            op = {"type": 0, "pos1": rnd.randint(0, length), "seg": "xy"}
            length += 2
        msgs.append(_msg(client, seq, seq - 1, op, msn))
    return init, msgs


def marker_batch(n_docs: int, n_ops: int, seed: int = 1, adjust: bool = False, docs=None, keep_messages=False,
                 wide: int = 0):
    """A batch of the generated documents (docs: the document indices to include, default all)."""
    b = MergeTreeStreamBuilder(keep_messages=keep_messages)
    for d in (range(n_docs) if docs is None else docs):
        init, msgs = doc_messages(d, n_ops, seed, adjust, wide)
        doc = b.begin_doc(init)
        for m in msgs:
            doc.add_message(m)
    return b.finish()
