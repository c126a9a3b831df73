# Quick GPU pass: parity tests, the dense single-gradient probe under rocprofv3, bench.
#   gpurun --timeout 900 -- 'bash tools/gpu_quick.sh <tag>'
set -e
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[quick] tests"
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "[quick] dense probe (rocprofv3)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_dense -o dense -- \
  python3 tools/dense_probe.py > $OUT/dense.log 2>&1
tail -1 $OUT/dense.log
find $OUT/prof_dense -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -12
if [ -z "$SKIP_BENCH" ]; then
echo "[quick] bench"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
fi
echo "[quick] done"
