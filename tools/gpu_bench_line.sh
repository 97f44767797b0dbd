#!/bin/bash
# Round 5: reduced T3 with the summary emission and the one-replay oracle check, then the default
# T1 bench line; every step time-limited and chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r5_bench}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --workload t3 --segments ${SEGS:-1000000} --t3-ops ${T3OPS:-200000} --steps 1 --warmup 1 --t3-check > $OUT/bench_T3.log 2>&1 \
 && timeout -k 10 400 python -u bench.py > $OUT/bench_T1.log 2>&1
rc=$?
tail -c 1500 $OUT/bench_T3.log; tail -c 600 $OUT/bench_T1.log
exit $rc
