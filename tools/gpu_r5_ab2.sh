#!/bin/bash
# Round 5: same-process A/B, second round — T1 (op-record loads through SGPR bases, 3 waves/SIMD)
# and T3 (window-pass and slot-pass unrolls), each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab2
mkdir -p $OUT
timeout -k 10 500 python3 tools/bench_variants.py --docs 20000 --unique 20000 --rounds 3 cur fetch_uni cw3 > $OUT/ab_t1.json 2> $OUT/ab_t1.err \
 && timeout -k 10 700 python3 tools/bench_variants.py --workload t3 --segments 2000000 --t3-ops 200000 --rounds 2 r5ck hcur pass4 shift8 > $OUT/ab_t3.json 2> $OUT/ab_t3.err
rc=$?
cat $OUT/ab_t1.json $OUT/ab_t3.json
exit $rc
