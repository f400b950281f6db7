#!/bin/bash
# rocprofv3 kernel trace (stats only) of a short bench run; prints the per-kernel averages.
# Usage (GPU box): bash tools/prof_quick.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-quick}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 "$@" > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/run.log; exit $rc; }
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:64]:64s} n={r["Calls"]:>4} avg={float(r["AverageNs"])/1e3:8.1f}us {float(r["TotalDurationNs"])/tot*100:5.1f}%')
PY
