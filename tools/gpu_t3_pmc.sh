#!/bin/bash
# T3 (hugeDocKernel) counters at this build on a slice (1M segments, 1e5 ops): the kernel trace, the
# instruction-cache hit/miss pass, and instruction-issue groups, one counter group per rocprofv3 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r6/t3_pmc}
mkdir -p $OUT
step() { echo "[$(date +%T)] $1" >> $OUT/progress.txt; }
D="python3 tools/pcs_driver.py --workload t3 --segments ${SEGS:-1000000} --t3-ops ${OPS:-100000} --runs 1 --lib fluidframework_amd/libfmt.so"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $D > $OUT/trace.log 2>&1 && step trace \
 && timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT/pmc_ic -o run -- $D > $OUT/pmc_ic.log 2>&1 && step icache \
 && timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES --output-format csv -d $OUT/pmc_insts -o run -- $D > $OUT/pmc_insts.log 2>&1 && step insts \
 && timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_cycles -o run -- $D > $OUT/pmc_cycles.log 2>&1 && step cycles
rc=$?
tail -3 $OUT/trace.log
exit $rc
