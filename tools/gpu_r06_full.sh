#!/bin/bash
# Round 6 record run: full GPU suite (parity report), smoke, default bench (with the CPU baseline),
# training benches (LightGlue, SuperGlue), the other BASELINE configs.
# usage (on the GPU box, from the repo root): bash tools/gpu_r06_full.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06_full}; mkdir -p $O
rm -f $O/parity_report.jsonl
LG_PARITY_REPORT=$O/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench.json; [ $rc -ne 0 ] && exit $rc
for w in train train_sg; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 5 --warmup 2 --cpu-budget 0 > $O/bench_$w.json 2> $O/bench_$w.err
  rc=$?; echo "bench $w rc=$rc $(python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print(d['value'], d['ms_per_step'])" 2>&1)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python3 tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err; rc=$?; echo "configs rc=$rc"; cut -c1-200 $O/configs.jsonl; [ $rc -ne 0 ] && exit $rc
exit 0
