#!/bin/bash
# New GPU tests (long inserts, huge tier) then the T1 scheduler-variant A/B, time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_long_inserts.py tests/test_huge_obliterate.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 900 python3 -u tools/bench_variants.py --docs 100000 --unique 100000 --rounds 3 "$@" > $OUT/ab_t1.json 2> $OUT/ab_t1.err
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/ab_t1.json 2>/dev/null
exit $rc
