#!/bin/bash
# Round 5: huge-tier variants at the plain-load build — graduation from one batched mask pass
# vs 4 — T3 slice, time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab15
mkdir -p $OUT
timeout -k 10 900 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 3 r5nb grad > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
