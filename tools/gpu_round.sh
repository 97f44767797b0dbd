#!/bin/bash
# GPU validation pass: parity tests (incl. the JavaScript driver), smoke, default bench (T1, all docs
# distinct) and the M2 map bench. Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 600 python bench.py > gpurun_out/bench_T1.log 2>&1 \
 && timeout -k 10 300 python bench.py --workload map > gpurun_out/bench_M2.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log 2>/dev/null; tail -1 gpurun_out/bench_T1.log 2>/dev/null | cut -c1-400
exit $rc
