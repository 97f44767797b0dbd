#!/bin/bash
# Round 6 diagnostics: the f4 local-client bench line (writer views of the reference farms), a T3
# A/B (per-phase clock reads on / off), and a PC-sampling pass over a T3 slice (line-table build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/diag}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
timeout -k 10 500 python3 -u bench.py --workload local --docs ${LDOCS:-20000} --steps 2 --warmup 1 --cpu-seconds 10 > $OUT/bench_local.log 2>&1 && step local \
 && OUT=$OUT WORKLOAD=t3 LIMIT=500 bash tools/gpu_ab_run.sh base t3noclk && step ab_t3 \
 && timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
      --pc-sampling-interval 1 --output-format csv -d $OUT/pcs_t3 -o run -- \
      python3 tools/pcs_driver.py --workload t3 --runs 1 > $OUT/pcs_t3.log 2>&1
rc=$?
step "pcs rc=$rc"
tail -1 $OUT/bench_local.log | cut -c1-2500
exit $rc
