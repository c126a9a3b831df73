# Round-4 pass F: the whole GPU suite with the in-kernel dense resolve (FC_DENSE_TAIL), then a
# same-box A/B (tail / no tail / direct packet entries) and the tail's phase trace.
#   gpurun --timeout 900 -- 'bash tools/r04_f.sh r04_f'
set -e
TAG=${1:-r04_f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 330 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 100 \
  --var tail= --var notail=tools/variants/lib_notail.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 134217728 --dense" \
  --probe "tools/sample_probe.py --n 16777216" --probe "tools/sample_probe.py --n 134217728"
for a in "--n 134217728 --dense" "--n 16777216 --dense"; do
  timeout -k 5 100 python tools/trace_probe.py --lib tools/variants/lib_trace.so $a >> $OUT/traces.jsonl
done
echo "[r04_f] done"
