set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_train.py --model superglue --batch 8 --npts 1024 --steps 3 --warmup 1 > gpurun_out/sgb_small.log 2>&1
rc=$?; echo small rc=$rc; tail -2 gpurun_out/sgb_small.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/bench_train.py --model superglue --steps 5 --warmup 2 > gpurun_out/sgb_c2.log 2>&1
rc=$?; echo c2 rc=$rc; tail -2 gpurun_out/sgb_c2.log; [ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/prof_sgtrain; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bench_train.py --model superglue --steps 2 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo trace rc=$rc; exit $rc
