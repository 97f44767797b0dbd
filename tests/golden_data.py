"""Loaders for the committed golden vectors in tests/golden/ (see tools/make_golden.py)."""
import json
import os

import numpy as np

from fluidframework_amd.streams import MergeTreeBatch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _js(a):
    return json.loads(a.tobytes().decode())


def replay_fixtures(bundle="replay_conflict_farm_0.40.npz"):
    """Yields (name, batch, group_end, initial_texts, result_texts) for the 30 fixtures of a bundle
    (the 0.40 conflict farms, or replay_obliterate_2.3.0.npz for the obliterate farms)."""
    z = np.load(os.path.join(GOLDEN, bundle), allow_pickle=False)
    names = _js(z["names"])
    for i, name in enumerate(names):
        ops = z[f"{i}/ops"]
        batch = MergeTreeBatch(
            ops=ops,
            doc_op_offsets=np.array([0, len(ops)], dtype=np.uint64),
            text=z[f"{i}/arena"],
            doc_init=z[f"{i}/doc_init"],
            props_off=z[f"{i}/props_off"],
            props_kv=z[f"{i}/props_kv"],
            keys=_js(z[f"{i}/keys_json"]),
            values=_js(z[f"{i}/values_json"]),
        )
        texts = _js(z[f"{i}/texts_json"])
        yield name, batch, z[f"{i}/group_end"], texts["initial"], texts["result"]


def prefix_batch(fixtures):
    """One document per (fixture, group): the fixture's ops up to the end of that group.

    Lets a single batched replay check every one of the 64 text checkpoints of every fixture.
    Returns (batch, expected_texts).
    """
    from fluidframework_amd.streams import MergeTreeStreamBuilder  # noqa: F401  (dtype owner)

    ops_list, offs, init, expected = [], [0], [], []
    texts, text_len = [], 0
    props_off_all, props_kv_all, n_props = [np.zeros(1, np.uint32)], [], 0
    keys, values = [], ["null"]
    for name, b, group_end, _, results in fixtures:
        # re-base this fixture's arena, props-op ids and dictionary ids into the combined batch
        ops = b.ops.copy()
        ins = ops["type"] == 0
        ops["payload"][ins] += text_len
        ann = ops["type"] == 2
        ops["payload"][ann] += n_props
        kmap = [_intern(keys, k) for k in b.keys]
        vmap = [0] + [_intern(values, v) for v in b.values[1:]]
        kv = np.array([(kmap[x >> 16] << 16) | vmap[x & 0xFFFF] for x in b.props_kv.tolist()], dtype=np.uint32)
        texts.append(b.text)
        init_off = b.doc_init[0].astype(np.int64)
        for g, end in enumerate(group_end):
            ops_list.append(ops[:end])
            offs.append(offs[-1] + int(end))
            init.append((int(init_off[0]) + text_len, int(init_off[1])))
            expected.append(results[g])
        text_len += len(b.text)
        props_off_all.append(b.props_off[1:].astype(np.int64) + int(props_off_all[-1][-1]))
        props_kv_all.append(kv)
        n_props += len(b.props_off) - 1
    batch = MergeTreeBatch(
        ops=np.concatenate(ops_list),
        doc_op_offsets=np.asarray(offs, dtype=np.uint64),
        text=np.concatenate(texts).astype("<u2"),
        doc_init=np.asarray(init, dtype=np.uint32),
        props_off=np.concatenate(props_off_all).astype(np.uint32),
        props_kv=np.concatenate(props_kv_all).astype(np.uint32),
        keys=keys,
        values=values,
    )
    return batch, expected


def _intern(lst, x):
    if x in lst:
        return lst.index(x)
    lst.append(x)
    return len(lst) - 1


def snapshot_trees(version="legacy"):
    with open(os.path.join(GOLDEN, f"snapshots_{version}.json")) as fh:
        return json.load(fh)
