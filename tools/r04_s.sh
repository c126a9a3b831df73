# Round-4 pass S: non-temporal packet entry / candidate stores (batched compaction, lone
# packet encode and its round trip), alternating builds.
set -e
OUT=gpurun_out/r04_s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var base= --var entnt=tools/variants/lib_entnt.so --var candnt=tools/variants/lib_candnt.so \
  --var bothnt=tools/variants/lib_bothnt.so \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10" --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10" \
  --probe "tools/single_diag.py --reps 2 --iters 30"
echo "[r04_s] done"
