#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE run separately).

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
  * both counters are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read, so it is
    doubled before it is compared with a byte count;
  * WRITE_SIZE is exact for 16-B-per-lane streaming stores (other widths are uncalibrated; the
    merge-tree's 4-32 B result stores are reported uncorrected).

Usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel substring>
       <workload key> <out json> [<lds counter_collection.csv>]
Env PMC_PER=<substring>: the dispatch that marks one run (e.g. CompactTier) when a run is several
dispatches of the kernel.
With the LDS pass (SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE) the record also carries the kernel's
LDS bank-conflict rate: conflict cycles / LDS-active cycles, summed over the launch's waves.
The output JSON maps a workload key (e.g. "mt:100000x2000") to the per-launch traffic record that
bench.py copies into its `roofline.traffic` field when it runs the same workload.
"""
import csv
import json
import os
import sys


def per_launch(path, kernel, counter, per=None):
    """Counter total per launch of the replay: summed over every dispatch whose name contains
    `kernel` (a run can be several dispatches: the compact tier, then the small tier over its
    overflow list), divided by the number of dispatches whose name contains `per` (one per run;
    default: `kernel`)."""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not rows:
        raise SystemExit(f"{path}: no {counter} rows for {kernel}")
    runs = len({r["Dispatch_Id"] for r in rows if (per or kernel) in r["Kernel_Name"]})
    return sum(float(r["Counter_Value"]) for r in rows) / max(runs, 1), runs


def main():
    fetch_csv, write_csv, kernel, key, out = sys.argv[1:6]
    per = os.environ.get("PMC_PER")
    f_kib, nf = per_launch(fetch_csv, kernel, "FETCH_SIZE", per)
    w_kib, nw = per_launch(write_csv, kernel, "WRITE_SIZE", per)
    rec = {
        "kernel": kernel,
        "fetch_bytes": f_kib * 1024 * 2,  # gfx950: FETCH_SIZE counts half of wide streaming reads
        "write_bytes": w_kib * 1024,
        "fetch_size_kib_raw": f_kib,
        "write_size_kib_raw": w_kib,
        "launches": [nf, nw],
        "source": [os.path.relpath(fetch_csv), os.path.relpath(write_csv)],
    }
    rec["bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
    if len(sys.argv) > 6:
        conf, _ = per_launch(sys.argv[6], kernel, "SQ_LDS_BANK_CONFLICT", per)
        act, _ = per_launch(sys.argv[6], kernel, "SQ_LDS_IDX_ACTIVE", per)
        rec["lds_bank_conflict_rate"] = conf / act if act else None
        rec["source"].append(os.path.relpath(sys.argv[6]))
    db = json.load(open(out)) if os.path.exists(out) else {}
    if "issue" in db.get(key, {}):
        rec["issue"] = db[key]["issue"]
    db[key] = rec
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
