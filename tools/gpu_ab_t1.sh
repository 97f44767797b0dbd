#!/bin/bash
# Same-process A/B of build/variants/* at the full T1 shape (100k documents x 2000 ops).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/bench_variants.py --docs ${DOCS:-100000} --unique ${DOCS:-100000} --rounds 3 "$@" > gpurun_out/ab_t1.json 2> gpurun_out/ab_t1.err
rc=$?
cat gpurun_out/ab_t1.json
exit $rc
