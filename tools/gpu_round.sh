# One GPU-box pass: parity tests, smoke, headline bench, rocprofv3 kernel stats, PMC HBM bytes.
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh <tag>'
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
N=134217728
K=13421773
if [ -z "$SKIP_TESTS" ]; then
echo "[gpu_round] tests"
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
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
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
if [ -z "$SKIP_PROF" ]; then
echo "[gpu_round] rocprofv3 kernel stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench -- \
  python3 bench.py --no-cpu-baseline --no-single > $OUT/prof_bench.log 2>&1
echo "[gpu_round] pmc FETCH_SIZE"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc -- \
  python3 tools/kbench.py --iters 3 --batch 4 --tag pmc > $OUT/pmc_fetch.log 2>&1
echo "[gpu_round] pmc WRITE_SIZE"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc -- \
  python3 tools/kbench.py --iters 3 --batch 4 --tag pmc > $OUT/pmc_write.log 2>&1
echo "[gpu_round] summaries"
python3 tools/rocpd_summary.py stats $(find $OUT/prof_bench -name "*.db" | head -1) \
  $OUT/kernel_stats_bench.csv
python3 tools/rocpd_summary.py pmc $(find $OUT/pmc_fetch -name "*.db" | head -1) \
  $(find $OUT/pmc_write -name "*.db" | head -1) k_compact_mag1 $OUT/pmc_k_compact_mag1.json \
  --alg-bytes $((4 * (4 * N + 8 * K))) --clients-per-launch 4
fi
echo "[gpu_round] done"
