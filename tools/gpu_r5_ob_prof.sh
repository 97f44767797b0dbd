#!/bin/bash
# Round 5: obliterate GPU tests, then the T1 compact tier's in-kernel phase profile (FMT_PROFILE=1
# build of build/variants/prof), each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_prof
K="obliterate or checkpoint or grow or huge or writer or capacity" OUTDIR=r5_ob bash tools/gpu_tests.sh
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python3 tools/mt_phase_profile.py --docs 20000 --unique 2000 > gpurun_out/r5_prof/phases_t1.txt 2>&1
