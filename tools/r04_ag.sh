# Round-4 pass AG: batched workspace stride (per-client workspaces padded by 4 / 12 / 64 KB).
set -e
OUT=gpurun_out/${1:-r04_ag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var new= --var sp4=tools/variants/lib_sp4.so --var sp12=tools/variants/lib_sp12.so \
  --var sp64=tools/variants/lib_sp64.so \
  --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10" --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10"
echo "[r04_ag] done"
