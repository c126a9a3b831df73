# Round-4 pass AN: the drop-in dense encode's sample size at 16 M (1/32 shipped; 1/64, 1/16).
set -e
OUT=gpurun_out/${1:-r04_an}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var dsd64=tools/variants/lib_dsd64.so --var dsd16=tools/variants/lib_dsd16.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 25557032 --dense --f 0.01" \
  --probe "tools/sample_probe.py --n 33554432 --dense"
echo "[r04_an] done"
