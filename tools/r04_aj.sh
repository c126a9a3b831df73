# Round-4 pass AJ: k_fold_q load-group size (items per group: 3 shipped, 2, 1) — the dense
# decode of ONE packet re-loads the same packet for every item slot of a group.
set -e
OUT=gpurun_out/${1:-r04_aj}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --out $OUT/ab.jsonl --reps 3 --timeout 150 \
  --var new= --var qg1=tools/variants/lib_qg1.so --var qg2=tools/variants/lib_qg2.so \
  --probe "tools/single_diag.py --reps 2 --iters 30 --n 134217728" --probe "tools/kbench.py --dec 128 --n 134217728 --iters 5"
echo "[r04_aj] done"
