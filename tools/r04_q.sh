# Round-4 pass Q: what the lone packet encode's post-bracket streaming pays for (ablation
# builds, results wrong by construction: timing only): no entry stores / no candidate stores /
# no per-chunk counts + shard atomics / none of them / loads only.
set -e
OUT=gpurun_out/r04_q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py --out $OUT/ab.jsonl --reps 2 --timeout 100 \
  --var base= --var noent=tools/variants/lib_noent.so --var nocand=tools/variants/lib_nocand.so \
  --var nometa=tools/variants/lib_nometa.so --var noall=tools/variants/lib_noall.so \
  --var loadonly=tools/variants/lib_loadonly.so \
  --probe "tools/sample_probe.py --n 134217728" --probe "tools/sample_probe.py --n 134217728 --dense"
echo "[r04_q] done"
