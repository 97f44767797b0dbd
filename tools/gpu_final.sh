#!/bin/bash
# End-of-round pass at HEAD: GPU parity suite, smoke, then one bench line per workload (T1 default,
# T2 slice, M2, M2 sparse with keys U[0, 2^20), T3 reduced, long documents, obliterate farms), each
# step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 \
 && step pytest \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
 && step smoke \
 && timeout -k 10 600 python bench.py > $OUT/bench_T1.log 2>&1 \
 && step T1 \
 && timeout -k 10 600 python bench.py --workload t2 --docs 40000 --steps 2 --gather-docs 64 > $OUT/bench_T2_slice.log 2>&1 \
 && step T2 \
 && timeout -k 10 600 python bench.py --workload map --steps 5 > $OUT/bench_M2.log 2>&1 \
 && step M2 \
 && timeout -k 10 600 python bench.py --workload map --sparse --key-pool 1048576 --steps 5 > $OUT/bench_M2_sparse.log 2>&1 \
 && step M2sparse \
 && timeout -k 10 600 python -u bench.py --workload t3 --segments 1000000 --t3-ops 200000 --steps 2 --warmup 1 --cpu-ops 100000 > $OUT/bench_T3_reduced.log 2>&1 \
 && step T3 \
 && timeout -k 10 600 python bench.py --min-length 3000 --docs 20000 --no-summaries --steps 2 > $OUT/bench_long_docs.log 2>&1 \
 && step long \
 && timeout -k 10 600 python bench.py --workload ob --steps 3 > $OUT/bench_ob.log 2>&1 \
 && step ob
rc=$?
tail -3 $OUT/pytest_gpu.log; for f in $OUT/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-200)"; done
exit $rc
