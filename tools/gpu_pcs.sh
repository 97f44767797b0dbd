#!/bin/bash
# Round 5: huge-tier / V1 loader GPU tests, a PC-sampling pass over a T1 slice (line-table build of
# the engine), then the T1 trace + PMC passes (tools/gpu_issue.sh); each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_pcs
K="huge or loader or v1_body or writer" OUTDIR=r5_huge bash tools/gpu_tests.sh
rc=$?
# (failed tests go on to the profiles; a time limit, abort or fault ends the call)
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 --output-format csv -d gpurun_out/r5_pcs/host_trap -o run -- \
  python3 tools/pcs_driver.py --docs 20000 --runs 1 > gpurun_out/r5_pcs/host_trap.log 2>&1
rc=$?
echo "pcs host_trap rc=$rc" >> gpurun_out/r5_pcs/host_trap.log
# (a time limit, abort or fault ends the call here; an unsupported option does not)
case $rc in 124|134|137|139) exit $rc ;; esac
OUTDIR=r5_issue_t1 bash tools/gpu_issue.sh
