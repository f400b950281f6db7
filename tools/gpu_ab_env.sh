# Same-box A/B of an environment setting (AB_ENV, e.g. "LG_LAYER_SLICES=0") against the default,
# after the training/gradient tests; two alternating rounds of tools/bench_train.py per model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sg_train.py tests/test_gpu_loss.py -q -s --timeout 150 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "worst|passed|failed|Error|assert" gpurun_out/ab_tests.log | cut -c1-200 | head -8; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ab_env.log
for round in 1 2; do
  for v in default "$AB_ENV"; do
    for model in ${AB_MODELS:-lightglue}; do
      if [ "$v" = default ]; then
        timeout -k 10 300 python -u tools/bench_train.py --model $model --steps 4 --warmup 2 > gpurun_out/ab_one.log 2>&1
      else
        timeout -k 10 300 env $v python -u tools/bench_train.py --model $model --steps 4 --warmup 2 > gpurun_out/ab_one.log 2>&1
      fi
      rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/ab_one.log; exit $rc; }
      echo "$round $v $model $(tail -1 gpurun_out/ab_one.log | cut -c1-220)" | tee -a gpurun_out/ab_env.log
    done
  done
done
