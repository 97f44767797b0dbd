#!/bin/bash
# Round 5 final (call B): full-size T3 (10M segments legacy load, 1e7 ops) with the summary emission
# and the one-replay oracle check (digest + summary + catch-up), one timed step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/${T3OUT:-r5_t3full}
timeout -k 10 1100 python -u bench.py --workload t3 --steps 1 --warmup 0 --t3-check > gpurun_out/${T3OUT:-r5_t3full}/bench_T3_full.log 2>&1
rc=$?
tail -c 3000 gpurun_out/${T3OUT:-r5_t3full}/bench_T3_full.log
exit $rc
