#!/bin/bash
# GPU parity suite, then a same-process A/B of build/variants (args) at full T1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-tests_ab}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 \
 && echo "[$(date +%T)] pytest" >> $OUT/progress.txt \
 && timeout -k 10 900 python3 -u tools/bench_variants.py --docs 100000 --unique 100000 --rounds 3 "$@" > $OUT/ab_t1.json 2> $OUT/ab_t1.err
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/ab_t1.json 2>/dev/null
exit $rc
