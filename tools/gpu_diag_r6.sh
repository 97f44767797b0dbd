#!/bin/bash
# Round 6 diagnostics: the f4 local-client bench line (writer views of the reference farms), a T3
# A/B (per-phase clock reads on / off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/diag}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 500 python3 -u bench.py --workload local --docs ${LDOCS:-20000} --steps 2 --warmup 1 --cpu-seconds 10 > $OUT/bench_local.log 2>&1 && step local \
 && OUT=$OUT WORKLOAD=t3 LIMIT=500 bash tools/gpu_ab_run.sh base t3noclk && step ab_t3
rc=$?
tail -1 $OUT/bench_local.log | cut -c1-2500
exit $rc
