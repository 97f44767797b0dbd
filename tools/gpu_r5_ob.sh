#!/bin/bash
# Round 5: obliterate GPU tests (HBM live-obliterate table in the huge tier, tiers escalating past 64
# live obliterates), time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
K="obliterate" OUTDIR=r5_ob bash tools/gpu_tests.sh
