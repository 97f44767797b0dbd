#!/bin/bash
# Full-size T3 (BASELINE config 5): 10M-segment SharedString, 1e7 ops, one timed step, CPU baseline sample.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u bench.py --workload t3 --steps 1 --warmup 0 "$@" > gpurun_out/bench_T3_full.log 2>&1
rc=$?
grep "phase\|step\|cpu" gpurun_out/bench_T3_full.log | cut -c1-400; tail -1 gpurun_out/bench_T3_full.log | cut -c1-3000
exit $rc
