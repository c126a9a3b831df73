# One GPU-box pass: parity tests, smoke, headline bench, rocprofv3 kernel stats (bench and the
# single-gradient dense path).  PMC passes: tools/pmc_round.sh.
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh <tag>'
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -e
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
echo "[gpu_round] tests"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "[gpu_round] smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
if [ -n "$E2E" ]; then
echo "[gpu_round] e2e"
timeout -k 10 300 python -u tools/e2e_bench.py > $OUT/e2e.json 2> $OUT/e2e.err
cat $OUT/e2e.json
fi
echo "[gpu_round] bench"
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
if [ -z "$SKIP_PROF" ]; then
echo "[gpu_round] rocprofv3 kernel stats (bench)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench -- \
  python3 bench.py --steps 10 --no-cpu-baseline --no-single > $OUT/prof_bench.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_bench -name "*.db" | head -1) \
  $OUT/kernel_stats_bench.csv
echo "[gpu_round] rocprofv3 kernel stats (single 128 M gradient, dense)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_dense -o dense -- \
  python3 tools/dense_probe.py > $OUT/prof_dense.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_dense -name "*.db" | head -1) \
  $OUT/kernel_stats_dense.csv
fi
echo "[gpu_round] done"
