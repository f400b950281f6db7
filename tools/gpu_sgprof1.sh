set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/prof_sgtrain4; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_train.py --model superglue --steps 2 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo sg trace rc=$rc; exit $rc
