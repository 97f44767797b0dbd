#!/bin/bash
# Round 5: window pass 2 x 64 + slot pass 4 x 64 (in-tree build) — the whole -m gpu suite, then the
# T3 slice A/B against the plain-load build; each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab11
mkdir -p $OUT
OUTDIR=r5_ab11 bash tools/gpu_tests.sh || exit $?
timeout -k 10 600 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 3 r5plain w2s4 > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
