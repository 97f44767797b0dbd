#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python3 tools/bench_variants.py --docs 20000 --unique 2000 --rounds 3 "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err
echo "exit $?"
