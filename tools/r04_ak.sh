# Round-4 pass AK: k_compact_mag1's client interleave (16 / 32 / 64 shipped / 128 clients) with
# the non-temporal packet stores.
set -e
OUT=gpurun_out/${1:-r04_ak}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var new= --var il16=tools/variants/lib_il16.so --var il32=tools/variants/lib_il32.so \
  --var il128=tools/variants/lib_il128.so \
  --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10" --probe "tools/kbench.py --batch 128 --n 134217728 --iters 5"
echo "[r04_ak] done"
