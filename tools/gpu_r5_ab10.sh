#!/bin/bash
# Round 5: huge-tier variants at the plain-load build — text reads as plain loads, slot-pass width 4,
# window-pass width 2 — T3 slice, time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab10
mkdir -p $OUT
timeout -k 10 900 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 2 r5plain ptext shift4b pass2b > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
