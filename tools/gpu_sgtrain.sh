set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg_train.py tests/test_gpu_superglue.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t_sgtrain.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|PASS|FAIL|worst|Error|error" gpurun_out/t_sgtrain.log | tail -30; exit $rc
