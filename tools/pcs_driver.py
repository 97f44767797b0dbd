#!/usr/bin/env python3
"""One T1-shaped (or --workload t3: T3-slice) replay through a given libfmt.so (a PC-sampling target: run under rocprofv3
--pc-sampling-*; tools/pcs_attribute.py maps the samples to source lines)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from fluidframework_amd import native, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "build/variants/lines/libfmt.so"))
    ap.add_argument("--docs", type=int, default=20000)
    ap.add_argument("--unique", type=int, default=2000)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--workload", choices=["mt", "t3"], default="mt")
    ap.add_argument("--segments", type=int, default=2_000_000, help="t3: segments of the loaded document")
    ap.add_argument("--t3-ops", type=int, default=200_000, help="t3: ops replayed")
    a = ap.parse_args()
    if a.workload == "t3":
        batch = workloads.t3_stream(a.segments, a.t3_ops)
    else:
        batch = workloads.conflict_farm(a.unique, n_clients=8, ops_per_doc=2000, seed=5, replicas=a.docs // a.unique)
    e = native.Engine(0, lib_path=a.lib)
    e.mt_load(batch)
    for k in range(a.runs):
        e.mt_run()
        e.sync()
        print(f"run {k}: {e.stats().kernel_ms:.1f} ms", flush=True)
    e.close()


if __name__ == "__main__":
    main()
