# Round-4 pass Y: histogram shard counts on the lone and batched encodes' latency chains —
# sample shards (max 8 / 4 / 2) and resolve candidate shards (4 / 2 / 8).
set -e
OUT=gpurun_out/${1:-r04_y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 120 \
  --var base= --var s2=tools/variants/lib_s2.so --var s1=tools/variants/lib_s1.so \
  --var c2=tools/variants/lib_c2.so --var c1=tools/variants/lib_c1.so \
  --var s2c2=tools/variants/lib_s2c2.so --var s1c1=tools/variants/lib_s1c1.so \
  --probe "tools/sample_probe.py --n 134217728" --probe "tools/sample_probe.py --n 134217728 --dense" \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10"
echo "[r04_y] done"
