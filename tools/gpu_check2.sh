#!/bin/bash
# Round-2 validation pass: GPU parity tests, smoke, T1 bench (3 steps), a small T2 bench on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py --steps 3 > gpurun_out/bench_T1.log 2>&1 \
 && timeout -k 10 600 python bench.py --workload t2 --docs 40000 --steps 2 --gather-docs 64 > gpurun_out/bench_T2_small.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log 2>/dev/null; tail -1 gpurun_out/bench_T1.log 2>/dev/null | cut -c1-600; tail -1 gpurun_out/bench_T2_small.log 2>/dev/null | cut -c1-300
exit $rc
