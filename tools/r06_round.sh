# Round-6 measurement pass (one GPU call): GPU suite, smoke, default bench, rocprofv3 kernel
# stats (bench step, lone round trip 128 M / 16 M, configs[1]/[2]), full-size Aggregator rates,
# and the k_compact_mag1 PMC traffic for the bench's roofline.
#   gpurun --timeout 1200 -- 'bash tools/r06_round.sh r06a'   (SKIP_TESTS=1 / SKIP_BENCH=1 /
#   SKIP_PROF=1 / SKIP_PMC=1 drop parts: two calls fit the 20-minute limit)
set -e
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
echo "[r06] tests"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
grep "GB/s" $OUT/gpu_tests.log || true
echo "[r06] smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
if [ -z "$SKIP_BENCH" ]; then
echo "[r06] bench"
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
fi
if [ -z "$SKIP_PROF" ]; then
echo "[r06] rocprofv3 kernel stats: bench step"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o bench -- \
  python3 bench.py --steps 10 --no-cpu-baseline --no-single > $OUT/prof_bench.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_bench -name "*.db" | head -1) $OUT/kernel_stats_bench.csv
echo "[r06] rocprofv3 kernel stats: lone round trip 128 M and 16 M"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lone -o lone -- \
  python3 tools/lone_probe.py > $OUT/prof_lone.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_lone -name "*.db" | head -1) $OUT/kernel_stats_lone.csv
echo "[r06] rocprofv3 kernel stats: configs[1]/[2]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c12 -o c12 -- \
  python3 tools/c2_probe.py --steps 50 > $OUT/prof_c12.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_c12 -name "*.db" | head -1) $OUT/kernel_stats_configs12.csv
echo "[r06] rocprofv3 kernel stats: native rand-k 16 M"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_randk -o rk -- \
  python3 tools/randk_probe.py > $OUT/prof_randk.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_randk -name "*.db" | head -1) $OUT/kernel_stats_randk.csv
fi
if [ -z "$SKIP_PMC" ]; then bash tools/pmc_round.sh ${TAG}_pmc; fi
echo "[r06] done"
