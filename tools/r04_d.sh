# Round-4 pass D: the whole GPU suite (QSGD quad decode, fp64, one-word window publication,
# adaptive histogram shards), QSGD probe, and a same-box A/B against the committed library and
# the lone-resolve grid variants.
#   gpurun --timeout 900 -- 'bash tools/r04_d.sh r04_d'
set -e
TAG=${1:-r04_d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for i in 1 2; do
  timeout -k 10 100 python tools/qsgd_probe.py --n 134217728 --tag qsgd$i >> $OUT/probes.jsonl
done
cat $OUT/probes.jsonl
timeout -k 10 400 python tools/ab.py --out $OUT/ab.jsonl --reps 1 --timeout 100 \
  --var new= --var head=tools/variants/lib_head.so --var base0=tools/variants/lib_base0.so \
  --var cpw32=tools/variants/lib_cpw32.so --var cpw16=tools/variants/lib_cpw16.so \
  --var drain1=tools/variants/lib_drain1.so --var drain2=tools/variants/lib_drain2.so \
  --var direct=tools/variants/lib_direct.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728" \
  --probe "tools/kbench.py --batch 64 --n 16777216"
echo "[r04_d] done"
