#!/bin/bash
# Map kernel iteration: map parity tests, M2 bench, kernel trace and FETCH/WRITE PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/map
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --workload map"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k map --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 \
 && timeout -k 10 300 $B --steps 5 --warmup 1 > $OUT/bench_M2.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_M2 -o run -- $B --steps 2 --warmup 1 > $OUT/trace_M2.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_M2 -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_fetch_M2.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_M2 -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_write_M2.log 2>&1
echo "exit $?"
