#!/bin/bash
# Same-process A/B of build/variants/* on a T3 slice (2M segments x 200k ops by default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/bench_variants.py --workload t3 --rounds 2 "$@" > gpurun_out/ab_t3.json 2> gpurun_out/ab_t3.err
rc=$?
cat gpurun_out/ab_t3.json; tail -3 gpurun_out/ab_t3.err
exit $rc
