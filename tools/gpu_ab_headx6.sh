set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIGHTGLUE_MI355X_LIB=$PWD/ab/headx6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 150 --timeout-method thread > gpurun_out/hx_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "worst|passed|failed" gpurun_out/hx_tests.log | cut -c1-300 | head -5
AB_LIBS=headx6.so bash tools/gpu_ab_train.sh
