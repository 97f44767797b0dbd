#!/usr/bin/env python3
"""Instruction-issue record of one kernel from rocprofv3 SQ/GRBM PMC passes (one counter group per run).

The merge-tree kernel is not bandwidth-bound: what limits it is how fast each SIMD
issues the instructions of its waves' dependent op chains. This turns the passes into per-op
instruction counts and the SIMD-cycle split bench.py reports beside the HBM fraction
(`roofline.issue`):
  * SQ_INSTS_* are wave-instructions summed over the launch;
  * SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md, "s_memtime
    tick vs SQ PMC units"), summed over waves; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ≈ WAVE_CYCLES;
  * GRBM_GUI_ACTIVE is the sum over the 8 XCDs of the busy GPU clock, so kernel cycles ≈ it ÷ 8;
  * VALU busy = 4 · ACTIVE_INST_VALU ÷ (kernel cycles × SIMDs): the fraction of all SIMD cycles in
    which a VALU instruction of this kernel was executing.

Usage: pmc_issue.py <kernel substring> <workload key> <ops per launch> <simds> <out json> <csv>...
The record is stored under db[key]["issue"] of the output JSON (profiles/traffic.json).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main():
    kernel, key, ops, simds, out = sys.argv[1:6]
    ops, simds = float(ops), int(simds)
    per = os.environ.get("PMC_PER") or kernel  # the dispatch that marks one run (see pmc_traffic.py)
    vals = defaultdict(float)
    runs = defaultdict(set)
    sources = []
    for path in sys.argv[6:]:
        sources.append(os.path.relpath(path))
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                name = r["Counter_Name"]
                vals[name] += float(r["Counter_Value"])
                if per in r["Kernel_Name"]:
                    runs[name].add((path, r["Dispatch_Id"]))  # GRBM_ sits in several passes
    c = {k: v / max(len(runs[k]), 1) for k, v in vals.items()}
    if not c:
        raise SystemExit(f"no rows for {kernel}")
    rec = {"kernel": kernel, "ops_per_launch": ops, "counters": c, "source": sources}
    per_op = {}
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                 "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"):
        if name in c:
            per_op[name[len("SQ_INSTS_"):].lower()] = c[name] / ops
    rec["insts_per_op"] = per_op
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        rec["wave_cycle_split"] = {k: c[n] / wc for k, n in (("active_inst_any", "SQ_ACTIVE_INST_ANY"),
                                                             ("wait_any", "SQ_WAIT_ANY"),
                                                             ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                                                             ("active_inst_valu", "SQ_ACTIVE_INST_VALU"),
                                                             ("active_inst_lds", "SQ_ACTIVE_INST_LDS"),
                                                             ("active_inst_sca", "SQ_ACTIVE_INST_SCA"))
                                   if n in c}
    grbm = [c[k] for k in c if k.startswith("GRBM_GUI_ACTIVE")]
    if grbm:
        cycles = grbm[0] / 8.0
        rec["kernel_cycles"] = cycles
        # Per-pipe busy fractions, each <= 1: a SIMD gets one issue slot per pipe every 4 cycles
        # (the sequencer visits the 4 SIMDs of a CU round-robin), and ACTIVE_INST_<pipe> counts the
        # quad-cycles in which that pipe held an instruction of this kernel. The pipes issue in
        # parallel, so the fractions do not add up to one "issue busy" figure.
        for pipe, n in (("valu", "SQ_ACTIVE_INST_VALU"), ("salu", "SQ_ACTIVE_INST_SCA"),
                        ("lds", "SQ_ACTIVE_INST_LDS")):
            if n in c:
                rec[f"{pipe}_busy"] = 4.0 * c[n] / (cycles * simds)
        if "SQ_BUSY_CYCLES" in c:
            rec["sq_busy_cycles"] = c["SQ_BUSY_CYCLES"]
    db = json.load(open(out)) if os.path.exists(out) else {}
    db.setdefault(key, {})["issue"] = rec
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps({k: v for k, v in rec.items() if k != "counters"}))


if __name__ == "__main__":
    main()
