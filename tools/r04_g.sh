# Round-4 pass G: QSGD probe (fp32 quantise), the integrated Aggregator's NumPy-to-NumPy rate,
# the k_compact_mag1 traffic refresh (PMC), and rocprofv3 kernel stats of the bench and of the
# single-gradient dense path.
#   gpurun --timeout 1190 -- 'bash tools/r04_g.sh r04_g'
set -e
TAG=${1:-r04_g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for i in 1 2; do
  timeout -k 10 100 python tools/qsgd_probe.py --n 134217728 --tag qsgd$i >> $OUT/probes.jsonl
done
cat $OUT/probes.jsonl
timeout -k 10 300 python -u -m pytest tests/test_fullsize_parity.py -x -q -s -m gpu -k "aggregator" \
  --timeout 280 --timeout-method thread > $OUT/aggregator.log 2>&1 || { tail -30 $OUT/aggregator.log; exit 1; }
grep "numpy->numpy" $OUT/aggregator.log
bash tools/pmc_round.sh $TAG/pmc_compact > $OUT/pmc_round.log 2>&1 || { tail -20 $OUT/pmc_round.log; exit 1; }
cat gpurun_out/$TAG/pmc_compact/pmc_k_compact_mag1.json
SKIP_TESTS=1 bash tools/gpu_round.sh $TAG > $OUT/round.log 2>&1 || { tail -20 $OUT/round.log; exit 1; }
tail -5 $OUT/round.log
echo "[r04_g] done"
