set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in train train_sg; do
  timeout -k 10 500 python -u bench.py --workload $w --steps 5 --warmup 2 > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; grep '^{' gpurun_out/bench_$w.log | cut -c1-600; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_$w.log; exit $rc; }
done
exit 0
