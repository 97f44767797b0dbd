#!/bin/bash
# Large-tier throughput: documents kept >= 3000 UTF-16 units (every one outgrows the small tier's 2048)
# — bench line with the CPU baseline, then the kernel trace of the same run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/large
mkdir -p $OUT
B="python3 bench.py --min-length 3000 --docs ${DOCS:-20000} --no-summaries"
timeout -k 10 600 $B --steps 2 --warmup 1 --cpu-seconds 10 > $OUT/bench_large.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 1 --warmup 0 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?
tail -1 $OUT/bench_large.log | cut -c1-1500
exit $rc
