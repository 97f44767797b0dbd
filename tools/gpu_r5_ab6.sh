#!/bin/bash
# Round 5: T3 A/B of the chunked group scan and the global-typed state pointers on a 10M-segment slice (1.5k groups, 2e5 ops), time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab6
mkdir -p $OUT
timeout -k 10 900 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 2 prev hcur gq > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t3.json
exit $rc
