#!/bin/bash
# LDS / issue counters for the attention kbench variants (one rocprofv3 pass per counter group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
export KB_ONLY="${KB_ONLY:-ping-pong}"
i=0
for ctr in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_attn/p$i" -- "$R/tools/kbench_attn" > "$R/gpurun_out/pmc_attn/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
