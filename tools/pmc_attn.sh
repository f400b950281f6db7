#!/bin/bash
# VALU / MFMA / LDS instruction counters for the attention micro-benchmark.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_attn; mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench_attn.hip -o /tmp/ka 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- /tmp/ka > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/b -o run -- /tmp/ka > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
echo done
