# Round-4 pass AA: one sample shard everywhere vs the shipped 2 (one per 128 workgroups).
set -e
OUT=gpurun_out/r04_aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var s1=tools/variants/lib_s1n.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 134217728 --dense" \
  --probe "tools/sample_probe.py --n 134217728"
echo "[r04_aa] done"
