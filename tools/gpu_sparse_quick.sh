#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/sp2
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "sparse" --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 \
 && timeout -k 10 300 python3 -u bench.py --workload map --sparse --key-pool 1048576 --steps 5 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; tail -1 $OUT/bench.log | cut -c1-600
exit $rc
