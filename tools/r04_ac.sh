# Round-4 pass AC: is the 16 M gain of one sample shard the code or the workspace layout?
# s1 (1 shard), s1pad (1 shard, layout of 2), s2pad (2 shards, layout of 3), new (2 shards).
set -e
OUT=gpurun_out/r04_ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 120 \
  --var new= --var s1=tools/variants/lib_s1n.so --var s1pad=tools/variants/lib_s1pad.so \
  --var s2pad=tools/variants/lib_s2pad.so \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216"
echo "[r04_ac] done"
