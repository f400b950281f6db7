#!/bin/bash
# Same-box A/B of library builds: bench.py alternating between the .so files given as arguments,
# ROUNDS times; one line per run (library, pairs/s, attention ms per launch, GEMM ms per step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "$@"; do
    LIGHTGLUE_MI355X_LIB=$(realpath "$lib") timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-budget 0 ${BENCH_ARGS:-} > gpurun_out/ab_run.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab_run.log; exit 1; }
    python3 - "$lib" <<'PY'
import json, sys
r = json.loads([l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][0])
k = r.get("kernels") or {}
print(f"{sys.argv[1]:28s} {r['value']:9.2f} pairs/s  attn {r['roofline']['avg_launch_ms']*1e3:7.1f} us  gemm {k.get('gemm_ms_per_step')} ms  assign {k.get('assign_ms_per_step')} ms", flush=True)
PY
  done
done
