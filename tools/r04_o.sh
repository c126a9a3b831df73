# Round-4 pass O: batched compaction efficiency against gradient length (128 clients, f = 0.1).
set -e
OUT=gpurun_out/r04_o
mkdir -p $OUT
export TMPDIR=/tmp
for n in 16777216 33554432 67108864 134217728 16777216; do
  timeout -k 10 200 python -u tools/kbench.py --batch 128 --n $n --iters 10 | tee -a $OUT/kb.jsonl
done
echo "[r04_o] done"
