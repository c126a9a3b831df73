# Round-4 pass AO: k_compact_mag1 / k_fused_mag at 6 or 7 waves per SIMD (more VGPRs, fewer
# SGPR spills) against 8.
set -e
OUT=gpurun_out/${1:-r04_ao}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var new= --var w6=tools/variants/lib_w6.so --var w7=tools/variants/lib_w7.so \
  --probe "tools/kbench.py --batch 64 --n 134217728 --iters 10" --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10" \
  --probe "tools/sample_probe.py --n 134217728" --probe "tools/sample_probe.py --n 134217728 --dense"
echo "[r04_ao] done"
