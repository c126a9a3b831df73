# Round-4 pass AH: lone k_resolve grid at 16 M (8 / 16 / 32 chunks per workgroup: 256 / 128 /
# 64 workgroups) — fewer workgroups, fewer ticket arrivals and histogram flushes.
set -e
OUT=gpurun_out/${1:-r04_ah}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var cpw16=tools/variants/lib_cpw16.so --var cpw32=tools/variants/lib_cpw32.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 25557032 --dense --f 0.01"
echo "[r04_ah] done"
