#!/bin/bash
# Round 5: obliterate workload A/B — the small tier saving its checkpoint after the op loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab13
mkdir -p $OUT
timeout -k 10 600 python3 tools/bench_variants.py --workload ob --docs 100000 --rounds 3 r5w2s4 obsb > $OUT/ab_ob.json 2> $OUT/ab_ob.err
rc=$?
cat $OUT/ab_ob.json
exit $rc
