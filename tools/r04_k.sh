# Round-4 pass K: kernel trace of configs[2] blocks with the batched encode on 2 streams
# (catch a slow block).
set -e
OUT=gpurun_out/${1:-r04_k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 tools/c2_diag.py --reps 8 --steps 60 --modes top2 > $OUT/diag.jsonl
cat $OUT/diag.jsonl
echo "[r04_k] done"
