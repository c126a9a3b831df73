# Batched compaction per client at 16 M vs 128 M (one stream, one launch each), and variants
# (tools/variants/lib_<V>.so) at 16 M.
set -e
timeout -k 5 120 python tools/kbench.py --batch 64 --n 16777216 --iters 10 --tag b64_16M
for V in ${VARS:-div16 div32}; do
  timeout -k 5 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch 64 --n 16777216 --iters 10 --tag b64_16M_$V
done
