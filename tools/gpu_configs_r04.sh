set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/configs_r04.jsonl 2> gpurun_out/configs_r04.err
rc=$?; echo configs rc=$rc; cut -c1-220 gpurun_out/configs_r04.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/configs_r04.err; exit $rc; }
bash tools/gpu_workloads.sh
