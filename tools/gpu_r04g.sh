set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 120 --timeout-method thread > gpurun_out/t_r04g.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|worst" gpurun_out/t_r04g.log | tail -4; [ $rc -gt 1 ] && exit $rc
for i in 1 2; do
for lib in default ab_t/occ1.so ab_t/occ1_bk32.so; do
  if [ $lib = default ]; then unset LIGHTGLUE_MI355X_LIB; else export LIGHTGLUE_MI355X_LIB=$PWD/$lib; fi
  echo "lib=$lib" >> gpurun_out/bt_r04g.log
  timeout -k 10 200 python -u tools/bench_train.py --steps 3 --warmup 1 2>&1 | grep metric >> gpurun_out/bt_r04g.log || exit 3
done
done
unset LIGHTGLUE_MI355X_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train_r04g -o run -- python3 tools/bench_train.py --steps 2 --warmup 1 > gpurun_out/prof_train_r04g.log 2>&1
echo prof rc=$?
cat gpurun_out/bt_r04g.log | cut -c1-200
