#!/bin/bash
# Round 5: T1 A/B of the zamboni scour changes (match classes and char offsets read lane-parallel,
# dropped text moved with register-resident offsets), each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab4
mkdir -p $OUT
timeout -k 10 600 python3 tools/bench_variants.py --docs 20000 --unique 20000 --rounds 4 cur visbf > $OUT/ab_t1.json 2> $OUT/ab_t1.err
rc=$?
cat $OUT/ab_t1.json
exit $rc
