#!/bin/bash
# Map path at this build: dense M2 (1M docs x 8 clients x 1k ops, 20-key pool) and
# sparse M2 (keys U[0, 2^20)): bench lines, kernel trace + stats, FETCH / WRITE / LDS PMC passes (one
# counter group per run), then per-launch traffic records into $OUT/traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/map}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
D="python3 bench.py --workload map --no-cpu-baseline"
S="python3 bench.py --workload map --sparse --key-pool 1048576 --no-cpu-baseline"
timeout -k 10 400 python3 -u bench.py --workload map --steps 10 --warmup 2 > $OUT/bench_M2.log 2>&1 && step bench_M2 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_M2 -o run -- $D --steps 5 --warmup 1 > $OUT/trace_M2.log 2>&1 && step trace_M2 \
 && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_M2 -o run -- $D --steps 1 --warmup 0 > $OUT/pmc_fetch_M2.log 2>&1 && step fetch_M2 \
 && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_M2 -o run -- $D --steps 1 --warmup 0 > $OUT/pmc_write_M2.log 2>&1 && step write_M2 \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_lds_M2 -o run -- $D --steps 1 --warmup 0 > $OUT/pmc_lds_M2.log 2>&1 && step lds_M2 \
 && timeout -k 10 400 python3 -u bench.py --workload map --sparse --key-pool 1048576 --steps 10 --warmup 2 > $OUT/bench_M2_sparse.log 2>&1 && step bench_sparse \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_M2_sparse -o run -- $S --steps 5 --warmup 1 > $OUT/trace_M2_sparse.log 2>&1 && step trace_sparse \
 && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_sparse -o run -- $S --steps 1 --warmup 0 > $OUT/pmc_fetch_sparse.log 2>&1 && step fetch_sparse \
 && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_sparse -o run -- $S --steps 1 --warmup 0 > $OUT/pmc_write_sparse.log 2>&1 && step write_sparse \
 && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_lds_sparse -o run -- $S --steps 1 --warmup 0 > $OUT/pmc_lds_sparse.log 2>&1 && step lds_sparse \
 && python3 tools/pmc_traffic.py $OUT/pmc_fetch_M2/run_counter_collection.csv $OUT/pmc_write_M2/run_counter_collection.csv mapLwwKernel map:1000000x1000 $OUT/traffic.json $OUT/pmc_lds_M2/run_counter_collection.csv \
 && python3 tools/pmc_traffic.py $OUT/pmc_fetch_sparse/run_counter_collection.csv $OUT/pmc_write_sparse/run_counter_collection.csv mapSparseKernel map:1000000x1000k1048576s $OUT/traffic.json $OUT/pmc_lds_sparse/run_counter_collection.csv
rc=$?
tail -1 $OUT/bench_M2.log | cut -c1-1200; tail -1 $OUT/bench_M2_sparse.log | cut -c1-1200
exit $rc
