set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_loss.py tests/test_gpu_superglue.py -q -s --timeout 120 --timeout-method thread > gpurun_out/train_check_$TAG.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|worst" gpurun_out/train_check_$TAG.log | tail -6
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/bench_train_$TAG.log 2>&1
echo train rc=$?; grep metric gpurun_out/bench_train_$TAG.log
