set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sg_train.py tests/test_gpu_loss.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_train_all.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/t_train_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/bt_lg.log 2>&1
rc=$?; echo lg rc=$rc; tail -1 gpurun_out/bt_lg.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --model superglue --steps 5 --warmup 2 > gpurun_out/bt_sg.log 2>&1
rc=$?; echo sg rc=$rc; tail -1 gpurun_out/bt_sg.log | cut -c1-300; exit $rc
