#!/bin/bash
# Round 5: the whole -m gpu suite at the plain-load huge-tier build, every test run (no -x), with the
# addon's SIGSEGV backtrace handler on (FMT_NAPI_BACKTRACE=1) for the node child processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export FMT_NAPI_BACKTRACE=1
OUT=gpurun_out/r5_plain2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
