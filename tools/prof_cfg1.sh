#!/bin/bash
# kernel-time sum vs wall time of configs[1] (B = 1, N = 1024): how much of a latency-shaped
# forward is launch gaps.  Usage (GPU box): bash tools/prof_cfg1.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_cfg1
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/bench_configs.py --only 1 --reps 20 > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; cat $OUT/run.log | tail -2
python3 - "$OUT/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 20 forwards: find gaps between consecutive kernels
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
n = len(ts)
tail = ts[-int(n * 0.45):]
busy = sum(e - s for s, e, _ in tail)
span = tail[-1][1] - tail[0][0]
print(f"kernels {len(tail)}, busy {busy/1e3:.1f} us, span {span/1e3:.1f} us, busy/span {busy/span:.3f}")
PY
