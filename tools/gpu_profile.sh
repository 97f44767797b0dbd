#!/bin/bash
# Full-size benches (T1 merge-tree, M2 map) plus rocprofv3 kernel-trace/stats and separate PMC passes
# (one counter group per run), then per-launch HBM traffic into gpurun_out/prof/traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 > $OUT/bench_T1.log 2>&1 \
 && timeout -k 10 600 python3 bench.py --workload map --steps 5 --warmup 1 > $OUT/bench_M2.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_T1 -o run -- $B --steps 2 --warmup 1 > $OUT/trace_T1.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_M2 -o run -- $B --workload map --steps 2 --warmup 1 > $OUT/trace_M2.log 2>&1 \
 && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_T1 -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_fetch_T1.log 2>&1 \
 && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_T1 -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_write_T1.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_M2 -o run -- $B --workload map --steps 1 --warmup 0 > $OUT/pmc_fetch_M2.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_M2 -o run -- $B --workload map --steps 1 --warmup 0 > $OUT/pmc_write_M2.log 2>&1 \
 && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_lds_T1 -o run -- $B --steps 1 --warmup 0 > $OUT/pmc_lds_T1.log 2>&1 \
 && python3 tools/pmc_traffic.py $OUT/pmc_fetch_T1/run_counter_collection.csv $OUT/pmc_write_T1/run_counter_collection.csv mergeTreeKernel mt:100000x2000 $OUT/traffic.json $OUT/pmc_lds_T1/run_counter_collection.csv \
 && python3 tools/pmc_traffic.py $OUT/pmc_fetch_M2/run_counter_collection.csv $OUT/pmc_write_M2/run_counter_collection.csv mapLwwKernel map:1000000x1000 $OUT/traffic.json
echo "exit $?"
