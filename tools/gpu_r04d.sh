set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r04d.log 2>&1
rc=$?; echo bench rc=$rc; tail -1 gpurun_out/bench_r04d.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/prof_train_r04d; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_train.py --steps 2 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo train-trace rc=$rc; [ $rc -ne 0 ] && { tail -5 $OUT/trace.log; exit $rc; }
bash tools/profile.sh r04d
