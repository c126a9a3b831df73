# Round-4 pass I: configs[2] bimodality — host enqueue vs GPU time, encode+decode vs the
# pipelined encode_fold_batch, 1 vs 2 streams, several processes.
set -e
OUT=gpurun_out/${1:-r04_i}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 120 python -u tools/c2_diag.py --reps 3 --steps 100 > $OUT/diag_$i.jsonl
  cat $OUT/diag_$i.jsonl
done
echo "[r04_i] done"
