set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_loss.py tests/test_gpu_parity.py -q -s --timeout 120 --timeout-method thread -k "train or loss or autograd or similarity or backward or head" > gpurun_out/t_r04i.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|worst|Error" gpurun_out/t_r04i.log | tail -6; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_train.py --steps 5 --warmup 2 2>&1 | grep metric | tee gpurun_out/bt_r04i.log
