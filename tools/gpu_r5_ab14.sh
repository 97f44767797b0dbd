#!/bin/bash
# Round 5: huge-tier variants at the plain-load build — window pass 1 x 64, slot pass 2 x 64
# vs 4 — T3 slice, time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab14
mkdir -p $OUT
timeout -k 10 900 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 3 r5nb pass1 shift2 > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
