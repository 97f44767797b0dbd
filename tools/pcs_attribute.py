#!/usr/bin/env python3
"""Attribute rocprofv3 PC samples (--pc-sampling-* CSV) to source lines and instruction classes.

Usage: pcs_attribute.py <pc_sampling csv> [--kernel SUBSTR] [--top N]
Prints, for the samples of the matching kernel dispatches: the share per instruction class (scalar
ALU s_*, vector ALU v_*, memory, LDS, branch, wait), the top source lines (from the instruction
comment that a -gline-tables-only build carries) and the top instructions. A sample is one wave's
PC at a host-trap tick, so shares are of wave time, stalls included."""
import argparse
import collections
import csv
import re
import sys


def classify(ins: str) -> str:
    op = ins.strip().split(" ")[0] if ins else ""
    if op.startswith("s_waitcnt") or op.startswith("s_wait"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch") or op.startswith("s_setpc") or op.startswith("s_swappc"):
        return "branch"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "vmem"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "lane-xfer"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--dispatches", default="", help="comma-separated dispatch ids to keep (default: all)")
    a = ap.parse_args()
    with open(a.csv, newline="") as f:
        rows = list(csv.DictReader(f))
    if not rows:
        sys.exit("no samples")
    cols = rows[0].keys()
    icol = next((c for c in cols if c.lower() == "instruction"), None)
    ccol = next((c for c in cols if "comment" in c.lower()), None)
    kcol = next((c for c in cols if "kernel" in c.lower() and "name" in c.lower()), None)
    dcol = next((c for c in cols if "dispatch" in c.lower()), None)
    keep = set(a.dispatches.split(",")) if a.dispatches else None
    sel = [r for r in rows if (not a.kernel or kcol is None or a.kernel in r.get(kcol, ""))
           and (keep is None or dcol is None or r.get(dcol) in keep)]
    print(f"{len(sel)} samples of {len(rows)} (columns: {', '.join(cols)})")
    cls = collections.Counter(classify(r.get(icol, "")) for r in sel)
    n = max(1, len(sel))
    print("\nby class:")
    for k, v in cls.most_common():
        print(f"  {k:10s} {v:8d} {100.0 * v / n:6.2f}%")
    lines = collections.Counter()
    for r in sel:
        c = r.get(ccol, "") if ccol else ""
        m = re.search(r"([\w./-]+\.(?:h|hip|cpp)):(\d+)", c)
        lines[f"{m.group(1).split('/')[-1]}:{m.group(2)}" if m else "?"] += 1
    print(f"\ntop {a.top} source lines:")
    for k, v in lines.most_common(a.top):
        print(f"  {k:32s} {v:8d} {100.0 * v / n:6.2f}%")
    ins = collections.Counter((r.get(icol, "") or "").split(" ")[0] for r in sel)
    print(f"\ntop {a.top} instructions:")
    for k, v in ins.most_common(a.top):
        print(f"  {k:32s} {v:8d} {100.0 * v / n:6.2f}%")
    by_line_cls = collections.defaultdict(collections.Counter)
    for r in sel:
        c = r.get(ccol, "") if ccol else ""
        m = re.search(r"([\w./-]+\.(?:h|hip|cpp)):(\d+)", c)
        key = f"{m.group(1).split('/')[-1]}:{m.group(2)}" if m else "?"
        by_line_cls[key][classify(r.get(icol, ""))] += 1
    print(f"\nsalu+branch samples by source line (top {a.top}):")
    sb = collections.Counter({k: v["salu"] + v["branch"] for k, v in by_line_cls.items()})
    for k, v in sb.most_common(a.top):
        print(f"  {k:32s} {v:8d} {100.0 * v / n:6.2f}%  {dict(by_line_cls[k])}")


if __name__ == "__main__":
    main()
