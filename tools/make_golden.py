#!/usr/bin/env python3
"""Convert the reference's own golden fixtures into compact vectors under tests/golden/.

Run in the build container (where /root/reference exists); the outputs are committed so the GPU
box and the CPU test suite never read /root/reference at run time.

Sources (data files held by the reference's own tests):
  packages/dds/merge-tree/src/test/results/*-default-conflict-farm-0.40.json
  packages/dds/merge-tree/src/test/results/*-conflict-farm-with-obliterate-2.3.0.json
      replayed by client.replay.spec.ts:20-76 (64 groups of {initialText, resultText, msgs, seq})
  packages/dds/sequence/src/test/snapshots/legacy/{headerOnly,headerAndBody,largeBody,withAnnotations,withMarkers}.json
      checked by snapshotVersion.spec.ts:146-170 ("Snapshot diff")

Outputs:
  replay_conflict_farm_0.40.npz   all 30 0.40 fixtures, packed by streams.py, with every checkpoint text
  replay_obliterate_2.3.0.npz     the 30 *-conflict-farm-with-obliterate-2.3.0 fixtures, the same way
  replay_msgs_0.40.json.gz        the raw sequenced messages (ISequencedDocumentMessage JSON exactly as the
                                  fixture holds them) of MSG_FILES, for the JavaScript driver's tests
  snapshots_legacy.json           the legacy SharedString summary trees
  snapshots_v1.json               the SnapshotV1 summary trees of the same strings (v1/*.json)
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from fluidframework_amd.streams import MT_OP_DTYPE, MergeTreeStreamBuilder  # noqa: E402

REF = "/root/reference/packages"
RESULTS = f"{REF}/dds/merge-tree/src/test/results"
SNAPSHOTS = f"{REF}/dds/sequence/src/test/snapshots/legacy"
SNAPSHOTS_V1 = f"{REF}/dds/sequence/src/test/snapshots/v1"
OUT = os.path.join(REPO, "tests", "golden")


def convert_replay(path: str) -> dict:
    groups = json.load(open(path))
    b = MergeTreeStreamBuilder()
    doc = b.begin_doc(initial_text=groups[0]["initialText"], observer="A")
    group_end = []
    result_texts = []
    initial_texts = []
    for g in groups:
        initial_texts.append(g["initialText"])
        for m in g["msgs"]:
            assert m["type"] == "op"
            doc.add_message(m)
        group_end.append(doc.n_ops)
        result_texts.append(g["resultText"])
    batch = b.finish()
    return {
        "ops": batch.ops,
        "arena": batch.text,
        "doc_init": batch.doc_init,
        "props_off": batch.props_off,
        "props_kv": batch.props_kv,
        "keys_json": np.frombuffer(json.dumps(batch.keys).encode(), dtype=np.uint8),
        "values_json": np.frombuffer(json.dumps(batch.values).encode(), dtype=np.uint8),
        "group_end": np.asarray(group_end, dtype=np.int64),
        "texts_json": np.frombuffer(
            json.dumps({"initial": initial_texts, "result": result_texts}).encode(), dtype=np.uint8
        ),
    }


MSG_FILES = [
    "len_1-clients_2-default-conflict-farm-0.40.json",
    "len_16-clients_4-default-conflict-farm-0.40.json",
    "len_64-clients_8-default-conflict-farm-0.40.json",
    "len_128-clients_8-default-conflict-farm-0.40.json",
    "len_256-clients_4-default-conflict-farm-0.40.json",
    "len_512-clients_8-default-conflict-farm-0.40.json",
]


def write_messages() -> None:
    import gzip

    out = []
    for f in MSG_FILES:
        groups = json.load(open(os.path.join(RESULTS, f)))
        out.append({"name": f, "groups": groups})
    with gzip.open(os.path.join(OUT, "replay_msgs_0.40.json.gz"), "wt", encoding="utf-8") as fh:
        json.dump(out, fh, separators=(",", ":"), ensure_ascii=False)


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    files = sorted(f for f in os.listdir(RESULTS) if f.endswith("-default-conflict-farm-0.40.json"))
    bundle = {}
    for i, f in enumerate(files):
        d = convert_replay(os.path.join(RESULTS, f))
        for k, v in d.items():
            bundle[f"{i}/{k}"] = v
    bundle["names"] = np.frombuffer(json.dumps(files).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "replay_conflict_farm_0.40.npz"), **bundle)
    files = sorted(f for f in os.listdir(RESULTS) if f.endswith("-conflict-farm-with-obliterate-2.3.0.json"))
    bundle = {}
    for i, f in enumerate(files):
        d = convert_replay(os.path.join(RESULTS, f))
        for k, v in d.items():
            bundle[f"{i}/{k}"] = v
    bundle["names"] = np.frombuffer(json.dumps(files).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "replay_obliterate_2.3.0.npz"), **bundle)
    write_messages()
    assert MT_OP_DTYPE.itemsize == 32

    n = write_snapshots()
    print(f"wrote {len(files)} replay fixtures and {n} snapshot trees to {OUT}")


SNAPSHOT_NAMES = ["headerOnly", "headerAndBody", "largeBody", "withAnnotations", "withMarkers"]


def write_snapshots():
    """The legacy and V1 summary trees (data files of the reference's tests, copied as JSON)."""
    snaps = {}
    for name in SNAPSHOT_NAMES:
        snaps[name] = json.load(open(os.path.join(SNAPSHOTS, name + ".json")))
    with open(os.path.join(OUT, "snapshots_legacy.json"), "w") as fh:
        json.dump(snaps, fh, separators=(",", ":"))
    write_v1_snapshots()
    return len(snaps)


def write_v1_snapshots():
    """sequence/src/test/snapshots/v1/*.json: SnapshotV1 summaries of the same detached strings
    (generateSharedStrings.ts with newMergeTreeSnapshotFormat), checked by snapshotVersion.spec.ts."""
    snaps = {}
    for name in SNAPSHOT_NAMES:
        snaps[name] = json.load(open(os.path.join(SNAPSHOTS_V1, name + ".json")))
    with open(os.path.join(OUT, "snapshots_v1.json"), "w") as fh:
        json.dump(snaps, fh, separators=(",", ":"))


if __name__ == "__main__":
    import sys

    if sys.argv[1:] == ["--snapshots-only"]:
        print(f"wrote {write_snapshots()} snapshot trees to {OUT}")
    else:
        main()
