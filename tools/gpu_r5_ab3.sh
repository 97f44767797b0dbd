#!/bin/bash
# Round 5: T3 pass-unroll A/B (third round), then the T2 bench at one rank through RCCL (--dist:
# torch.distributed nccl initialised, the stats all-gather and summary gatherv over RCCL), each step
# time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5_ab3
mkdir -p $OUT
timeout -k 10 700 python3 tools/bench_variants.py --workload t3 --segments 2000000 --t3-ops 200000 --rounds 2 r5ck hcur pass2 shift4 > $OUT/ab_t3.json 2> $OUT/ab_t3.err \
 && timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
      bench.py --gpus 1 --workload t2 --docs 40000 --dist --steps 2 --warmup 1 --no-cpu-baseline --no-js-baseline > $OUT/bench_T2_rccl.log 2>&1
rc=$?
cat $OUT/ab_t3.json; tail -c 1500 $OUT/bench_T2_rccl.log
exit $rc
