#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUTDIR=issue_t1_r3 bash tools/gpu_issue.sh || exit $?
timeout -k 10 300 python3 tools/mt_phase_profile.py --lib build/variants/prof/libfmt.so > gpurun_out/issue_t1_r3/phases.json 2> gpurun_out/issue_t1_r3/phases.err
