set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sg_train.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_ab_train.log 2>&1
rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/t_ab_train.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ab_train.log
for round in 1 2; do
  for lib in default ${AB_LIBS:-x6off.so}; do
    if [ "$lib" != default ]; then export LIGHTGLUE_MI355X_LIB=$PWD/ab/$lib; else unset LIGHTGLUE_MI355X_LIB; fi
    for model in lightglue superglue; do
      timeout -k 10 300 python -u tools/bench_train.py --model $model --steps 4 --warmup 2 > gpurun_out/ab_one.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/ab_one.log; exit $rc; }
      echo "$round $lib $model $(tail -1 gpurun_out/ab_one.log | cut -c1-200)" | tee -a gpurun_out/ab_train.log
    done
  done
done
