set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ${KB_LIBS:-default}; do
  if [ "$lib" != default ]; then export LIGHTGLUE_MI355X_LIB=$PWD/ab/$lib; else unset LIGHTGLUE_MI355X_LIB; fi
  OUT=gpurun_out/kb_tgemm_$lib; mkdir -p $OUT
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/kbench_tgemm.py > $OUT/log 2>&1
  rc=$?; echo "$lib rc=$rc"; grep "rel err" $OUT/log | head -3; [ $rc -ne 0 ] && { tail -5 $OUT/log; exit $rc; }
done
[ -n "${KB_PMC:-}" ] && bash tools/pmc_cmd.sh tgemm python3 tools/kbench_tgemm.py
exit 0
