#!/bin/bash
# rocprofv3 kernel trace + stats of one tools/bench_configs.py config; prints the per-kernel
# averages and the busy/span ratio of the last forwards.  Usage (GPU box): bash tools/prof_cfg.sh <config#> [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${1:-1}; REPS=${2:-20}
OUT=gpurun_out/prof_cfg$C
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_configs.py --only $C --reps $REPS > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 $OUT/run.log
[ $rc -ne 0 ] && exit $rc
python3 - "$OUT/run_kernel_trace.csv" "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
tail = ts[-int(len(ts) * 0.45):]
busy = sum(e - s for s, e, _ in tail)
span = tail[-1][1] - tail[0][0]
print(f"kernels {len(tail)}, busy {busy/1e3:.1f} us, span {span/1e3:.1f} us, busy/span {busy/span:.3f}")
st = list(csv.DictReader(open(sys.argv[2])))
tot = sum(float(r["TotalDurationNs"]) for r in st)
for r in sorted(st, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{r["Name"][:70]:70s} n={r["Calls"]:>5} avg={float(r["AverageNs"])/1e3:8.1f}us {float(r["TotalDurationNs"])/tot*100:5.1f}%')
PY
