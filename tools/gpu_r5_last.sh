#!/bin/bash
# Round 5, last check of the committed tree: the whole -m gpu suite and smoke(), time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_last
mkdir -p $OUT
OUTDIR=r5_last bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?
tail -2 $OUT/smoke.log
exit $rc
