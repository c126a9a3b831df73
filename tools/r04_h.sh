# Round-4 pass H: configs[1]/[2] alone (tools/c2_probe.py), current library vs the committed
# round-4 baseline library, twice in alternating order.
set -e
TAG=${1:-r04_h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 120 \
  --var new= --var head=tools/variants/lib_head.so --probe "tools/c2_probe.py --steps 100"
cat $OUT/ab.jsonl
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -c 3000 $OUT/bench.json
echo "[r04_h] done"
