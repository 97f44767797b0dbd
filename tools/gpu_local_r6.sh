#!/bin/bash
# Round 6: local batches in the register tiers — the f4 GPU tests, an A/B of the local tier paths
# (compact → large, small → large, compact → small → large), the local bench line at 100k documents
# and its kernel trace; then the huge-tier GPU tests and a T3 A/B of the window table's LDS mirror
# (prev = HEAD~'s hugedoc, cur = this tree's).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/local2}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 600 python3 -u -m pytest tests/test_local_client.py tests/test_local_spec.py -m gpu -x -v \
    --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_local.log 2>&1 && step pytest \
 && OUT=$OUT WORKLOAD=local LIMIT=400 bash tools/gpu_ab_run.sh locCL locSL locCSL && step ab \
 && timeout -k 10 500 python3 -u bench.py --workload local --steps 3 --warmup 1 --cpu-seconds 20 > $OUT/bench_local_100k.log 2>&1 && step bench100k \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_local -o run -- \
      python3 bench.py --workload local --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace_local.log 2>&1 && step trace \
 && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_huge.py tests/test_huge_checkpoint.py tests/test_obliterate_ceiling.py tests/test_writer_ceiling.py -m gpu -x -v \
    --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_huge.log 2>&1 && step pytest_huge \
 && OUT=$OUT WORKLOAD=t3 LIMIT=500 bash tools/gpu_ab_run.sh prev cur && step ab_t3
rc=$?
tail -3 $OUT/pytest_local.log; tail -1 $OUT/bench_local_100k.log | cut -c1-1500
exit $rc
