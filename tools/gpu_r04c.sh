set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs4.py tests/test_gpu_loss.py tests/test_gpu_parity.py -k "configs4 or similarity or sinkhorn or autograd" -q -s --timeout 120 --timeout-method thread > gpurun_out/t_r04c.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed|configs4:" gpurun_out/t_r04c.log | tail -5
[ $rc -gt 1 ] && exit $rc
SK_SETTINGS=0:1:0,0:1:64,0:1:128,0:1:160,0:1:192,0:1:224,0:1:0,0:1:128,0:1:192 timeout -k 10 500 python -u tools/sk_sweep.py > gpurun_out/sk_r04c.log 2>&1
cat gpurun_out/sk_r04c.log | grep group
