#!/bin/bash
# Round 5: the whole -m gpu suite, then the reduced T3 (summary + oracle check) and the default T1
# bench line (tools/gpu_r5_bench.sh); each step time-limited, a fault or time limit ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUTDIR=r5_full bash tools/gpu_tests.sh
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
OUTDIR=r5_full bash tools/gpu_r5_bench.sh
