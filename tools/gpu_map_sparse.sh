#!/bin/bash
# Sparse SharedMap path on the GPU: parity tests, then M2 with keys U[0, 2^20) (bench + rocprof stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_map_sparse
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sparse" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_map_sparse.log 2>&1 \
 && timeout -k 10 400 python -u bench.py --workload map --sparse --key-pool 1048576 --steps 5 > gpurun_out/bench_M2_sparse.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_map_sparse -o run -- python -u bench.py --workload map --sparse --key-pool 1048576 --steps 5 > gpurun_out/rocprof_map_sparse.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_map_sparse.log; tail -1 gpurun_out/bench_M2_sparse.log | cut -c1-1500
exit $rc
