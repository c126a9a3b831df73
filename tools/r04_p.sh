# Round-4 pass P: the fused kernel's bracket poll — one word (base) vs a longer sleep vs
# 16 / 64 replicated publication lines; FC_TRACE phase timelines of base vs 64 copies.
set -e
OUT=gpurun_out/r04_p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 100 \
  --var base= --var s16=tools/variants/lib_s16.so --var c64=tools/variants/lib_c64.so \
  --var c16=tools/variants/lib_c16.so \
  --probe "tools/sample_probe.py --n 134217728" --probe "tools/sample_probe.py --n 134217728 --dense" \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216"
for V in trace trace_c64; do
  for a in "--n 134217728" "--n 16777216 --dense"; do
    timeout -k 5 100 python tools/trace_probe.py --lib tools/variants/lib_$V.so $a | sed "s/^{/{\"v\": \"$V\", /" >> $OUT/traces.jsonl
  done
done
echo "[r04_p] done"
