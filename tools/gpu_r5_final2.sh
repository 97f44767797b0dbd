#!/bin/bash
# Round 5 final, second build (global-typed huge state, heap sifts): the whole -m gpu suite, smoke(), the default T1 bench line, then the T1
# kernel trace + HBM traffic + instruction-issue PMC passes (tools/gpu_issue.sh); each step
# time-limited, a fault or time limit ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_final2
mkdir -p $OUT
OUTDIR=r5_final2 bash tools/gpu_tests.sh
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
 && timeout -k 10 400 python3 -u bench.py > $OUT/bench_T1.log 2>&1 \
 && OUTDIR=r5_final2/issue_t1 bash tools/gpu_issue.sh
