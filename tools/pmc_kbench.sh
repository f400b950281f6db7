#!/bin/bash
# SQ/GRBM counters for the kernel micro-benchmarks (MFMA busy, waits, clock).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_kb; mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I cs566-project-lightglue_amd/csrc tools/kbench_gemm.hip -o /tmp/kb 2>/dev/null || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench_attn.hip -o /tmp/ka 2>/dev/null || exit 1
for prog in kb ka; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$prog -o run -- /tmp/$prog > $OUT/$prog.log 2>&1 || { echo "$prog failed"; tail -5 $OUT/$prog.log; exit 1; }
done
echo done
