# Round-4 pass AE: workspace-region offsets (8 KB pads before hist1 / tick / status / cand,
# 4 KB before cand) against the shipped layout, on the lone packet/dense encodes and the
# batched compaction.
set -e
OUT=gpurun_out/${1:-r04_ae}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 150 \
  --var new= --var ph=tools/variants/lib_ph.so --var pt=tools/variants/lib_pt.so \
  --var ps=tools/variants/lib_ps.so --var pc=tools/variants/lib_pc.so --var pc4=tools/variants/lib_pc4.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728" \
  --probe "tools/kbench.py --batch 128 --n 16777216 --iters 10"
echo "[r04_ae] done"
