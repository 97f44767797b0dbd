#!/bin/bash
# Round 5: hole-moving heap sifts (both children in one LDS round trip) vs HEAD — T1 slice, obliterate
# workload, T3 slice; each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab8
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_variants.py --workload mt --docs 40000 --rounds 5 r5gq heap2 > $OUT/ab_t1.json 2> $OUT/ab_t1.err && cat $OUT/ab_t1.json &&
timeout -k 10 300 python3 tools/bench_variants.py --workload ob --docs 100000 --rounds 3 r5gq heap2 > $OUT/ab_ob.json 2> $OUT/ab_ob.err && cat $OUT/ab_ob.json &&
timeout -k 10 600 python3 tools/bench_variants.py --workload t3 --segments 10000000 --t3-ops 200000 --rounds 2 r5gq heap2 > $OUT/ab_t3.json 2> $OUT/ab_t3.err && cat $OUT/ab_t3.json
