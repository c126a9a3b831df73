# Round-4 pass E: the whole GPU suite on the sample-chain changes (one-word window publication,
# adaptive histogram shards), then a same-box A/B against the committed library and the
# lone-resolve grid variants.
#   gpurun --timeout 1190 -- 'bash tools/r04_e.sh r04_e'
set -e
TAG=${1:-r04_e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 100 \
  --var new= --var head=tools/variants/lib_head.so --var base0=tools/variants/lib_base0.so \
  --var cpw32=tools/variants/lib_cpw32.so --var cpw16=tools/variants/lib_cpw16.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728" \
  --probe "tools/kbench.py --batch 64 --n 16777216"
echo "[r04_e] done"
