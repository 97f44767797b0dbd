#!/bin/bash
# Sparse SharedMap path on the GPU: parity tests, then M2 with keys U[0, 2^20): bench line (with the
# CPU baseline), kernel trace + stats, FETCH/WRITE/LDS-conflict PMC passes (one counter group per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-map_sparse}
mkdir -p $OUT
B="python3 bench.py --workload map --sparse --key-pool 1048576 --no-cpu-baseline"
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "sparse" --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_map_sparse.log 2>&1 \
 && step pytest \
 && timeout -k 10 400 python3 -u bench.py --workload map --sparse --key-pool 1048576 --steps 5 > $OUT/bench_M2_sparse.log 2>&1 \
 && step bench \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_M2_sparse -o run -- $B --steps 2 --warmup 1 > $OUT/trace.log 2>&1 \
 && step trace \
 && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_fetch.log 2>&1 \
 && step fetch \
 && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_write.log 2>&1 \
 && step write \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_lds -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_lds.log 2>&1 \
 && step lds
rc=$?
tail -3 $OUT/pytest_map_sparse.log; tail -1 $OUT/bench_M2_sparse.log | cut -c1-1500
exit $rc
