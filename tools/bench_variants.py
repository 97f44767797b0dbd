#!/usr/bin/env python3
"""Same-process A/B timing of libfmt.so variants (build/variants/*/libfmt.so) on one batch.

Interleaves variants over rounds (cdna_hip_programming.md §5.4 rule 24) and checks every variant's
per-document headers against the in-tree library's."""
import argparse
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from fluidframework_amd import native, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=20000)
    ap.add_argument("--unique", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", choices=["mt", "map", "t3", "ob", "local"], default="mt")
    ap.add_argument("--segments", type=int, default=2_000_000, help="t3: segments of the loaded document")
    ap.add_argument("--t3-ops", type=int, default=200_000, help="t3: ops replayed")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    paths = {os.path.basename(os.path.dirname(p)): p for p in glob.glob(os.path.join(REPO, "build/variants/*/libfmt.so"))}
    if a.variants:
        paths = {k: v for k, v in paths.items() if k in a.variants}
    if a.workload == "map":
        return bench_map(a, paths)
    if a.workload == "t3":
        batch = workloads.t3_stream(a.segments, a.t3_ops)
    elif a.workload == "local":  # f4 writer views of the reference farms cycled to --docs (bench.py local)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from local_farm import fixture_local_docs

        batch = workloads.replicate_batches([f[1] for f in fixture_local_docs()], a.docs)
    elif a.workload == "ob":  # the reference's obliterate farms cycled to --docs documents (bench.py ob)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from golden_data import replay_fixtures

        batch = workloads.replicate_batches([f[1] for f in replay_fixtures("replay_obliterate_2.3.0.npz")], a.docs)
    else:
        batch = workloads.conflict_farm(a.unique, n_clients=8, ops_per_doc=2000, seed=5, replicas=a.docs // a.unique)
    ref = native.Engine(0)
    ref.mt_load(batch)
    ref.mt_run()
    ref_h = ref.mt_headers()
    ref.close()
    engines = {}
    for name, p in sorted(paths.items()):
        e = native.Engine(0, lib_path=p)
        e.mt_load(batch)
        e.mt_run()
        h = e.mt_headers()
        ok = all(np.array_equal(h[f], ref_h[f]) for f in ("status", "n_leaves", "n_chars", "n_blocks", "visible_len", "min_seq"))
        engines[name] = (e, ok)
    times = {k: [] for k in engines}
    for _ in range(a.rounds):
        for name, (e, _) in engines.items():
            e.mt_run()
            times[name].append(e.stats().kernel_ms)
    n_ops = len(batch.ops)
    out = {name: {"ok": ok, "ms": times[name], "min_ms": min(times[name]), "mops": n_ops / min(times[name]) / 1e3,
                  "launches": int(e.stats().launches)}
           for name, (e, ok) in engines.items()}
    print(json.dumps(out))


def bench_map(a, paths):
    batch = workloads.map_stream(a.docs, 1000, key_pool=20, seed=5)
    ref = native.Engine(0)
    ref.map_load(batch)
    ref.map_run()
    ref_s = ref.map_fetch()
    ref.close()
    engines = {}
    for name, p in sorted(paths.items()):
        print(f"[ab] {name}", file=sys.stderr, flush=True)
        e = native.Engine(0, lib_path=p)
        e.map_load(batch)
        e.map_run()
        e.sync()
        engines[name] = (e, bool(np.array_equal(e.map_fetch(), ref_s)))
    times = {k: [] for k in engines}
    for _ in range(a.rounds):
        for name, (e, _) in engines.items():
            e.map_run()
            times[name].append(e.stats().kernel_ms)
    n_ops = len(batch.ops)
    out = {name: {"ok": ok, "ms": times[name], "min_ms": min(times[name]), "gops": n_ops / min(times[name]) / 1e6,
                  "gbps": n_ops * 16.16 / min(times[name]) / 1e6}
           for name, (e, ok) in engines.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
