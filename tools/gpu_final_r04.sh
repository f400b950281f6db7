# Round-end record: smoke, every GPU test, the headline bench, both training benches, and a
# rocprofv3 kernel-stats pass over each training step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LG_PARITY_REPORT=gpurun_out/parity_report.jsonl bash tools/gpu_round.sh || exit $?
bash tools/gpu_bench_train.sh || exit $?
export TMPDIR=/tmp
for m in lightglue superglue; do
  OUT=gpurun_out/prof_train_$m; mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_train.py --model $m --steps 2 --warmup 1 > $OUT/trace.log 2>&1
  rc=$?; echo "$m trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
