# Round-4 pass AD: candidate-slot stride skew (the 16 M dense encode's 4-5 us depends on the
# workspace layout: s1pad/s2pad in r04_ac) — 0 / 8 / 16 / 32 extra entries per slot.
set -e
OUT=gpurun_out/${1:-r04_ad}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var cp2=tools/variants/lib_cp2.so --var cp4=tools/variants/lib_cp4.so --var cp8=tools/variants/lib_cp8.so \
  --var cp16=tools/variants/lib_cp16.so --var s2pad=tools/variants/lib_s2pad.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728"
echo "[r04_ad] done"
