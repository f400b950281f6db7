#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (HBM bytes) for the bench workload.
# Usage (on the GPU box): bash tools/profile.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-budget 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/trace.log; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/fetch.log; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/write.log; exit $rc; }
find $OUT -name "*.csv" | head -20
