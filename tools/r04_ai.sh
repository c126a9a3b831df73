# Round-4 pass AI: the encoder state block's offset in the workspace (0 / 4 / 8 / 16 KB).
set -e
OUT=gpurun_out/${1:-r04_ai}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var new= --var st4=tools/variants/lib_st4.so --var st8=tools/variants/lib_st8.so \
  --var st16=tools/variants/lib_st16.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728" \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10"
echo "[r04_ai] done"
