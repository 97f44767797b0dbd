#!/bin/bash
# GPU parity tests on the in-tree library, then interleaved A/B of build/variants/*, then the
# per-phase profile of the prof variant (if built). Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python3 tools/bench_variants.py --docs 20000 --unique 2000 --rounds 3 "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err \
 && { [ ! -f build/variants/prof/libfmt.so ] || timeout -k 10 300 python3 tools/mt_phase_profile.py > gpurun_out/phases.json 2> gpurun_out/phases.err; }
echo "exit $?"
