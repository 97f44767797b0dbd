#!/bin/bash
# Quick T3 timing: reduced T3 bench (1M segments, 100k ops) with the phase clocks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_huge.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_huge.log 2>&1 \
 && timeout -k 10 400 python -u bench.py --workload t3 --segments 1000000 --t3-ops 100000 --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/bench_T3_quick.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_huge.log; grep "phase\|step" gpurun_out/bench_T3_quick.log
exit $rc
