# Round-4 pass AF: candidate binning in the fused launch (one device atomic per candidate) vs
# in the resolve, re-measured with the candidate histogram's padded offset: packet path with
# in-kernel binning (pktbin), dense path binning in the resolve (densebin0).
set -e
OUT=gpurun_out/${1:-r04_af}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var pktbin=tools/variants/lib_pktbin.so --var densebin0=tools/variants/lib_densebin0.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/sample_probe.py --n 134217728 --dense" --probe "tools/sample_probe.py --n 134217728"
echo "[r04_af] done"
