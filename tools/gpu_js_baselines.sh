#!/bin/bash
# Bench lines carrying the JS worker_threads baselines next to the C++ oracle: T1 (default), long
# documents, M1; each step time-limited and chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-js}
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_T1.log 2>&1 \
 && timeout -k 10 600 python bench.py --min-length 3000 --docs 20000 --no-summaries --steps 2 > $OUT/bench_long_docs.log 2>&1 \
 && timeout -k 10 300 python bench.py --workload map --docs 1000 --clients 4 --steps 5 > $OUT/bench_M1.log 2>&1
rc=$?
for f in $OUT/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-300)"; done
exit $rc
