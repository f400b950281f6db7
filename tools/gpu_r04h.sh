set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 120 --timeout-method thread > gpurun_out/t_r04h.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|worst|Error" gpurun_out/t_r04h.log | tail -6; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
for lib in default ab_t/occ1.so; do
  if [ $lib = default ]; then unset LIGHTGLUE_MI355X_LIB; else export LIGHTGLUE_MI355X_LIB=$PWD/$lib; fi
  echo "lib=$lib" >> gpurun_out/bt_r04h.log
  timeout -k 10 200 python -u tools/bench_train.py --steps 3 --warmup 1 2>&1 | grep metric >> gpurun_out/bt_r04h.log || exit 3
done
done
cat gpurun_out/bt_r04h.log | cut -c1-220
