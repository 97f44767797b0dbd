#!/bin/bash
# T3 validation pass: huge-document GPU parity tests first, then the whole GPU suite, then a reduced
# T3 bench (1M segments, 100k ops) with the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_huge.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_huge.log 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python -u bench.py --workload t3 --segments 1000000 --t3-ops 200000 --steps 2 --warmup 1 --cpu-ops 100000 > gpurun_out/bench_T3_small.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_huge.log; tail -3 gpurun_out/pytest_gpu.log 2>/dev/null; tail -3 gpurun_out/bench_T3_small.log 2>/dev/null | cut -c1-900
exit $rc
