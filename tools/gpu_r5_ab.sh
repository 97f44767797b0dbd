#!/bin/bash
# Round 5: same-process A/B of build/variants — T1 (compact-tier chars moves) and T3 (huge-tier heap
# and window-pass variants) — each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab
mkdir -p $OUT
timeout -k 10 500 python3 tools/bench_variants.py --docs 20000 --unique 20000 --rounds 3 cur shift4 > $OUT/ab_t1.json 2> $OUT/ab_t1.err \
 && timeout -k 10 600 python3 tools/bench_variants.py --workload t3 --segments 2000000 --t3-ops 200000 --rounds 2 r5ck hcur pass8 > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t1.json $OUT/ab_t3.json
exit $rc
