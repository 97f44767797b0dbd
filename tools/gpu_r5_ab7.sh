#!/bin/bash
# Round 5: obliterate workload A/B — the cascade's small tier at 2 vs 1 waves/SIMD (spills vs AGPRs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab7
mkdir -p $OUT
timeout -k 10 600 python3 tools/bench_variants.py --workload ob --docs 100000 --rounds 3 ob_base ob_o1 > $OUT/ab_ob.json 2> $OUT/ab_ob.err
rc=$?
cat $OUT/ab_ob.json
exit $rc
