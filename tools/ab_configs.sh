#!/bin/bash
# Same-box A/B of library builds on the other configs: tools/bench_configs.py --only $ONLY
# alternating between the .so files given as arguments, ROUNDS times (one JSON line per run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    echo "== $lib"
    LIGHTGLUE_MI355X_LIB=$(realpath "$lib") timeout -k 10 300 python tools/bench_configs.py --only ${ONLY:-1} --reps ${REPS:-10} 2>&1 | grep '^{' | cut -c1-220 || { echo "$lib failed"; exit 1; }
  done
done
