"""Documents that grow past the large tier's 2048 leaves / 131,071 UTF-16 units from an empty or short
start: sequenced message streams for the stream builder.

Writers insert U[20, 60]-unit runs at random positions, remove up to 12 units and annotate small
ranges. Most messages are caught up (refSeq = seq - 1); one in four lags by up to `lag` seqs (never
behind the writer's own last message), with its positions inside the length every client saw at its
refSeq — which is that op's whole view, since its writer has nothing unacked. minSeq trails seq by
`window`.
"""
import random


def growth_messages(n_ops=4000, writers=6, lag=40, window=64, seed=1, initial=""):
    rnd = random.Random(seed)
    msgs = []
    hist = [len(initial)]  # visible length after each seq (index = seq)
    last = {}
    for seq in range(1, n_ops + 1):
        c = f"w{rnd.randrange(writers)}"
        ref = seq - 1
        if rnd.random() < 0.25 and seq > lag + 2:
            ref = max(seq - 1 - rnd.randrange(lag), last.get(c, 0))
        view, length = hist[ref], hist[-1]
        r = rnd.random()
        if r < 0.8 or view < 40:
            n = rnd.randint(20, 60)
            op = {"pos1": rnd.randint(0, view), "seg": "".join(rnd.choice("abcdefghij") for _ in range(n)), "type": 0}
        elif r < 0.93:
            a = rnd.randint(0, view - 13)
            op = {"pos1": a, "pos2": a + rnd.randint(1, 12), "type": 1}
        else:
            a = rnd.randint(0, view - 9)
            op = {"pos1": a, "pos2": a + rnd.randint(1, 8), "props": {"k": rnd.randrange(5)}, "type": 2}
        msgs.append({"clientId": c, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                     "minimumSequenceNumber": max(0, seq - window), "type": "op", "contents": op})
        last[c] = seq
        if op["type"] == 0:
            length += len(op["seg"])
        elif op["type"] == 1:
            length = _recount(initial, msgs) if ref != seq - 1 else length - (op["pos2"] - op["pos1"])
        hist.append(length)
    return msgs


def _recount(initial, msgs):
    """Visible length after msgs, from the oracle (a lagging remove may overlap concurrent ones)."""
    import oracle

    from fluidframework_amd.streams import MergeTreeStreamBuilder

    b = MergeTreeStreamBuilder()
    d = b.begin_doc(initial, observer="observer")
    for m in msgs:
        d.add_message(m)
    rc, h, *_ = oracle.mt_replay_batch(b.finish(), cap_leaves=1 << 16, cap_chars=1 << 19, cap_props=1024)
    assert rc == 0
    return int(h[0]["visible_len"])


def growth_batch(specs):
    """specs: [(initial text, n_ops, seed)] -> MergeTreeBatch, one document each."""
    from fluidframework_amd.streams import MergeTreeStreamBuilder

    b = MergeTreeStreamBuilder()
    for initial, n_ops, seed in specs:
        d = b.begin_doc(initial, observer="observer")
        for m in growth_messages(n_ops=n_ops, seed=seed, initial=initial):
            d.add_message(m)
    return b.finish()
