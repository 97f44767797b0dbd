#!/bin/bash
# Round 6 final check at this build: the whole -m gpu suite, smoke(), the default T1 bench line and
# the local-client bench line at 100k documents; every step time-limited and chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/final}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 && step pytest \
 && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 && step smoke \
 && timeout -k 10 300 python3 -u bench.py > $OUT/bench_T1.log 2>&1 && step bench_T1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log; tail -1 $OUT/bench_T1.log | cut -c1-300
exit $rc
