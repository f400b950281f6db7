set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs4.py tests/test_gpu_loss.py tests/test_gpu_parity.py -k "configs4 or similarity or sinkhorn or autograd" -v -s --timeout 120 --timeout-method thread > gpurun_out/t_r04b.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|configs4:" gpurun_out/t_r04b.log | tail -5
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  SK_SETTINGS=0:1 timeout -k 10 200 python -u tools/sk_sweep.py >> gpurun_out/sk_r04b.log 2>&1 || exit 3
  SK_SETTINGS=0:1 LIGHTGLUE_MI355X_LIB=$PWD/ab_sk/sk_log2_0.so timeout -k 10 200 python -u tools/sk_sweep.py >> gpurun_out/sk_r04b.log 2>&1 || exit 3
done
SK_SETTINGS=1:2,2:2,3:3,4:2,2:4 timeout -k 10 400 python -u tools/sk_sweep.py >> gpurun_out/sk_r04b.log 2>&1
cat gpurun_out/sk_r04b.log | grep group
