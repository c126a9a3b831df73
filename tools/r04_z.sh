# Round-4 pass Z: 2 sample shards (one per 128 sample workgroups) + 2 candidate shards against
# the previous library (8 adaptive / 4), alternating; then the GPU suite.
set -e
OUT=gpurun_out/r04_z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 150 \
  --var new= --var head=tools/variants/lib_head.so \
  --probe "tools/single_diag.py --reps 2 --iters 30" --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10" \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10" --probe "tools/f64_probe.py"
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "[r04_z] done"
