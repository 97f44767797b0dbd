#!/bin/bash
# Same-process A/B of build/variants/<name>/libfmt.so (tools/build_variants.py) on the GPU box,
# time-limited. Replaces the per-experiment gpu_r5_ab*.sh scripts of round 5.
#
#   OUT=gpurun_out/<dir> WORKLOAD=mt|t3|ob|local|map [ARGS="..."] [LIMIT=seconds] tools/gpu_ab_run.sh <variant>...
#
# WORKLOAD defaults to mt (a T1 slice: 20k distinct documents); t3 defaults to a 2M-segment / 2e5-op
# slice (ARGS="--segments 10000000" for the full document); ob cycles the reference's obliterate farms.
# The JSON (per-variant times, headers equal to the in-tree library's) goes to $OUT/ab_<workload>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-mt}
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
case $W in
  mt) DEF="--docs 20000 --unique 20000 --rounds 3" ;;
  t3) DEF="--workload t3 --segments 2000000 --t3-ops 200000 --rounds 2" ;;
  ob) DEF="--workload ob --docs 100000 --rounds 3" ;;
  local) DEF="--workload local --docs 20000 --rounds 3" ;;
  map) DEF="--workload map --rounds 5" ;;
  *) echo "unknown WORKLOAD $W" >&2; exit 2 ;;
esac
timeout -k 10 "${LIMIT:-600}" python3 -u tools/bench_variants.py $DEF ${ARGS:-} "$@" > "$OUT/ab_$W.json" 2> "$OUT/ab_$W.err"
rc=$?
cat "$OUT/ab_$W.json"; tail -3 "$OUT/ab_$W.err"
exit $rc
