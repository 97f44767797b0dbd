#!/bin/bash
# Counter list, then the instruction-cache hit/miss PMC pass at T1 (one short run), time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-icache}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o "SQC_[A-Z_]*" $OUT/counters.txt | sort -u > $OUT/sqc.txt
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT/pmc_ic -o run -- python3 bench.py --no-cpu-baseline --no-summaries --steps 1 --warmup 0 > $OUT/pmc_ic.log 2>&1
rc=$?
cat $OUT/sqc.txt | tr '\n' ' '; echo; tail -2 $OUT/pmc_ic.log
exit $rc
