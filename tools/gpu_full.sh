#!/bin/bash
# Full GPU check of the tree: the -m gpu suite, smoke, and the default bench line.
# usage (on the GPU box, from the repo root): bash tools/gpu_full.sh <tag>
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo bench failed; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
