#!/bin/bash
# Same-box A/B of environment settings on one library: bench.py alternating between the settings
# given as arguments (each a space-separated VAR=value list, "" for none), ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for setting in "$@"; do
    env $setting timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-budget 0 ${BENCH_ARGS:-} > gpurun_out/ab_run.log 2>&1 || { echo "[$setting] failed"; tail -5 gpurun_out/ab_run.log; exit 1; }
    python3 - "$setting" <<'PY'
import json, sys
r = json.loads([l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][0])
k = r.get("kernels") or {}
print(f"[{sys.argv[1]:24s}] {r['value']:9.2f} pairs/s  attn {r['roofline']['avg_launch_ms']*1e3:7.1f} us  gemm {k.get('gemm_ms_per_step')} ms", flush=True)
PY
  done
done
