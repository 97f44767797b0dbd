#!/bin/bash
# T1 merge-tree kernel at HEAD: same-process A/B of build/variants (20k docs), then the full-size
# kernel trace, HBM traffic (FETCH_SIZE / WRITE_SIZE) and the instruction-issue PMC passes, one
# counter group per run; every step time-limited and chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-issue}
mkdir -p $OUT
W=${W:-}  # workload arguments (default T1), e.g. W="--workload ob"
B="python3 bench.py $W --no-cpu-baseline --no-summaries --steps 1 --warmup 0"
AB=${AB:-}
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
step start
if [ -n "$AB" ]; then
  timeout -k 10 500 python3 tools/bench_variants.py --docs 20000 --unique 20000 --rounds 3 $AB > $OUT/ab.json 2> $OUT/ab.err || exit $?
  step ab
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_T1 -o run -- python3 bench.py $W --no-cpu-baseline --no-summaries --steps 2 --warmup 1 > $OUT/trace_T1.log 2>&1 \
 && step trace \
 && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1 \
 && step fetch \
 && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1 \
 && step write \
 && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_lds -o run -- $B > $OUT/pmc_lds.log 2>&1 \
 && step lds \
 && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_i1 -o run -- $B > $OUT/pmc_i1.log 2>&1 \
 && step i1 \
 && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_i2 -o run -- $B > $OUT/pmc_i2.log 2>&1 \
 && step i2
rc=$?
cat $OUT/ab.json 2>/dev/null
exit $rc
