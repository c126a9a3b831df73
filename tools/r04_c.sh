# Round-4 pass C: QSGD / fp64 parity after the arithmetic changes, their probes, the lone
# fused-encode PMC (packet vs dense) and the k_compact_mag1 traffic refresh.
#   gpurun --timeout 1190 -- 'bash tools/r04_c.sh r04_c'
set -e
TAG=${1:-r04_c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_f64_boundary.py -x -q -m gpu \
  -k "qsgd or f64" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 100 python tools/qsgd_probe.py --n 134217728 --tag qsgd$i >> $OUT/probes.jsonl
  timeout -k 10 100 python tools/f64_probe.py --n 16777216 --tag f64_$i >> $OUT/probes.jsonl
  timeout -k 10 100 python tools/sample_probe.py --n 134217728 --tag pkt$i >> $OUT/probes.jsonl
  timeout -k 10 100 python tools/sample_probe.py --n 134217728 --dense --tag dense$i >> $OUT/probes.jsonl
done
cat $OUT/probes.jsonl
bash tools/pmc_fused.sh $TAG/pmc_fused > $OUT/pmc_fused.log 2>&1 || { tail -20 $OUT/pmc_fused.log; exit 1; }
tail -3 $OUT/pmc_fused.log
bash tools/pmc_round.sh $TAG/pmc_compact > $OUT/pmc_round.log 2>&1 || { tail -20 $OUT/pmc_round.log; exit 1; }
cat gpurun_out/$TAG/pmc_compact/pmc_k_compact_mag1.json
echo "[r04_c] done"
