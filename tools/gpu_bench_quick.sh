#!/bin/bash
# GPU tests + default bench line (T1) + map bench line, each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python3 bench.py > gpurun_out/bench_T1.log 2>&1 \
 && timeout -k 10 600 python3 bench.py --workload map > gpurun_out/bench_M2.log 2>&1
echo "exit $?"
