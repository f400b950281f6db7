set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg_train.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t_sgtrain2.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|worst|Error" gpurun_out/t_sgtrain2.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/bench_train.py --model superglue --steps 5 --warmup 2 > gpurun_out/sgb_c2b.log 2>&1
rc=$?; echo c2 rc=$rc; tail -1 gpurun_out/sgb_c2b.log; [ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/prof_sgtrain2; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_train.py --model superglue --steps 2 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo trace rc=$rc; exit $rc
