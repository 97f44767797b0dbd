#!/bin/bash
# Same-process A/B of build/variants/* on the T1-shaped workload, then the phase profile variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/bench_variants.py --docs 20000 --unique 20000 --rounds 3 "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err \
 && timeout -k 10 300 python3 tools/mt_phase_profile.py --docs 20000 --unique 20000 > gpurun_out/phases.json 2> gpurun_out/phases.err
rc=$?
cat gpurun_out/ab.json
exit $rc
