# Training/gradient tests with the worst-ratio printout, then the same-box A/B of tools/gpu_ab_train.sh
# against the libraries named in AB_LIBS (ab/*.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sg_train.py tests/test_gpu_loss.py -q -s --timeout 150 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "worst|passed|failed|Error|assert" gpurun_out/ab_tests.log | cut -c1-260 | head -20; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_train.sh
