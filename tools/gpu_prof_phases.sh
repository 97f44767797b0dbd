#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/mt_phase_profile.py "$@" > gpurun_out/phases.json 2> gpurun_out/phases.err
echo "exit $?"
