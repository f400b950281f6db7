#!/bin/bash
# SQ counters of the bench workload for both fp16x3 attention kernels (h3g / h3m), one PMC pass
# per counter group, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0"
for K in h3m h3g; do
  OUT=gpurun_out/pmc_ab_$K; mkdir -p $OUT
  LG_ATTN_KERNEL=$K timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- python3 bench.py $ARGS > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
  LG_ATTN_KERNEL=$K timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o run -- python3 bench.py $ARGS > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
done
head -6 gpurun_out/pmc_ab_h3m/summary.txt; head -6 gpurun_out/pmc_ab_h3g/summary.txt
