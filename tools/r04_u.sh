# Round-4 pass U: paired-item batched compaction (the second item's loads issued before the
# first item's stores; 16 / 12 / 8 of its 16 loads per lane prefetched) against the one-item
# workgroup.
set -e
OUT=gpurun_out/r04_u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var base= --var pair16=tools/variants/lib_pair16.so --var pair12=tools/variants/lib_pair12.so \
  --var pair8=tools/variants/lib_pair8.so \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10" --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10"
echo "[r04_u] done"
