#!/bin/bash
# Same-process A/B of build/variants/* at full T1 (args: variant names), then the phase profile of
# build/variants/${PROF:-prof}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/bench_variants.py --docs ${DOCS:-100000} --unique ${DOCS:-100000} --rounds 3 "$@" > gpurun_out/ab_t1.json 2> gpurun_out/ab_t1.err || exit $?
cat gpurun_out/ab_t1.json
timeout -k 10 300 python3 tools/mt_phase_profile.py --lib build/variants/${PROF:-prof}/libfmt.so > gpurun_out/phases.json 2> gpurun_out/phases.err || exit $?
cat gpurun_out/phases.json
