# Round-4 pass L: batched encodes serialized per device — configs[2] blocks (2-stream mode
# must no longer stall), then the full round pass (tests, smoke, bench, kernel stats).
set -e
OUT=gpurun_out/r04_l
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/c2_diag.py --reps 4 --steps 100 --modes top2,top1,fold2 > $OUT/diag_$i.jsonl
  cat $OUT/diag_$i.jsonl
done
bash tools/gpu_round.sh r04_l
