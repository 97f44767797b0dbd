#!/bin/bash
# Obliterate workload: the reference's 30 obliterate conflict farms cycled to 100k documents —
# bench line with the CPU baseline, then the kernel trace of the same run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-ob}
mkdir -p $OUT
B="python3 bench.py --workload ob --docs ${DOCS:-100000}"
timeout -k 10 600 $B --steps ${STEPS:-3} --warmup 1 --cpu-seconds 10 > $OUT/bench_ob.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 1 --warmup 0 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?
tail -1 $OUT/bench_ob.log | cut -c1-1800
exit $rc
