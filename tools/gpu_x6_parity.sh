set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in default x6dgrad.so; do
  if [ "$lib" != default ]; then export LIGHTGLUE_MI355X_LIB=$PWD/ab/$lib; else unset LIGHTGLUE_MI355X_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sg_train.py -q -s --timeout 150 --timeout-method thread -k "backward or training_step or ragged" > gpurun_out/x6p_$lib.log 2>&1
  rc=$?; echo "$lib pytest rc=$rc"; grep -E "worst|passed|failed" gpurun_out/x6p_$lib.log | cut -c1-300
  [ $rc -gt 1 ] && exit $rc
done
exit 0
