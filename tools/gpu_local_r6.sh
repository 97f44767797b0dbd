#!/bin/bash
# Round 6: local batches in the compact tier — the f4 GPU tests, the local bench line (20k and 100k
# documents), an A/B of the compact local variant at 3 vs 2 waves/SIMD, and the kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/local}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 600 python3 -u -m pytest tests/test_local_client.py tests/test_local_spec.py tests/test_napi.py -m gpu -x -v \
    --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_local.log 2>&1 && step pytest \
 && timeout -k 10 300 python3 -u bench.py --workload local --docs 20000 --steps 3 --warmup 1 --cpu-seconds 10 > $OUT/bench_local_20k.log 2>&1 && step bench20k \
 && timeout -k 10 500 python3 -u bench.py --workload local --steps 3 --warmup 1 --cpu-seconds 20 > $OUT/bench_local_100k.log 2>&1 && step bench100k \
 && OUT=$OUT WORKLOAD=local LIMIT=400 bash tools/gpu_ab_run.sh loc3 loc2 && step ab \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_local -o run -- \
      python3 bench.py --workload local --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace_local.log 2>&1 && step trace
rc=$?
tail -3 $OUT/pytest_local.log; tail -1 $OUT/bench_local_100k.log | cut -c1-1500
exit $rc
