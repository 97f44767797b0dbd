#!/bin/bash
# Round 5: the huge-tier and V1 loader GPU tests, then the T1 trace + PMC passes (tools/gpu_issue.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_huge
K="huge or loader or v1_body" OUTDIR=r5_huge bash tools/gpu_tests.sh \
 && OUTDIR=r5_issue_t1 bash tools/gpu_issue.sh
