#!/bin/bash
# One validation pass at the working tree: GPU parity suite, smoke, T1 bench (with the summaries and
# catch-up records), M2 sparse bench, and a T3 slice (10M segments, 300k ops: the full document's
# index sizes), each step time-limited; OUTDIR names the directory under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-pass}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 \
 && step pytest \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && step smoke \
 && timeout -k 10 600 python -u bench.py > $OUT/bench_T1.log 2>&1 \
 && step T1 \
 && timeout -k 10 300 python -u bench.py --workload map --sparse --key-pool 1048576 --steps 5 --no-cpu-baseline > $OUT/bench_M2_sparse.log 2>&1 \
 && step M2sparse \
 && timeout -k 10 600 python -u bench.py --workload t3 --segments 10000000 --t3-ops 300000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_T3_slice.log 2>&1 \
 && step T3
rc=$?
tail -3 $OUT/pytest_gpu.log; for f in $OUT/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-250)"; done
exit $rc
