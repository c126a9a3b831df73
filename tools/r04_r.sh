# Round-4 pass R: the batched compaction's cost structure (ablation builds, timing only):
# 64 x 128 M and 128 x 16 M, base / no stores / loads only / no entry stores.
set -e
OUT=gpurun_out/r04_r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var base= --var noall=tools/variants/lib_noall.so --var loadonly=tools/variants/lib_loadonly.so \
  --var noent=tools/variants/lib_noent.so \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10" --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10"
echo "[r04_r] done"
