#!/bin/bash
# Round 5: huge tier HBM reads as plain loads vs workgroup-scope atomic loads (T3 slice), time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab9
mkdir -p $OUT
timeout -k 10 600 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 2 r5heap plainrd > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
