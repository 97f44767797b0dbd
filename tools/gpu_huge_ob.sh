#!/bin/bash
# Huge-tier GPU tests (obliterates, growth, T3 parity) and a T3 slice, time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-huge_ob}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_huge_obliterate.py tests/test_gpu_huge.py tests/test_growth.py tests/test_v1_body_load.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 \
 && timeout -k 10 600 python -u bench.py --workload t3 --segments 10000000 --t3-ops 300000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_T3_slice.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; for f in $OUT/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-250)"; done
exit $rc
