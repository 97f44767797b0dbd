#!/bin/bash
# Round 6 check at this build: the whole -m gpu suite, a T3 A/B of the huge-tier changes (prev =
# HEAD~'s hugedoc, cur = the LDS window mirror, t3lat = mirror + count/flag loads beside the leaf
# fields), the local bench line at 100k documents (small tier first) and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/check}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 && step pytest \
 && OUT=$OUT WORKLOAD=t3 LIMIT=600 bash tools/gpu_ab_run.sh prev cur t3lat && step ab_t3 \
 && timeout -k 10 500 python3 -u bench.py --workload local --steps 3 --warmup 1 --cpu-seconds 20 > $OUT/bench_local_100k.log 2>&1 && step bench_local \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_local -o run -- \
      python3 bench.py --workload local --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace_local.log 2>&1 && step trace_local
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/bench_local_100k.log | cut -c1-600
exit $rc
