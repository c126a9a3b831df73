# Batched compaction (one stream, one launch) of the default build and variants
# (tools/variants/lib_<V>.so): B clients x N (defaults 64 x 16 M).
set -e
N=${N:-16777216}; B=${B:-64}
timeout -k 5 120 python tools/kbench.py --batch $B --n $N --iters ${IT:-10} --tag b${B}_$N
for V in ${VARS:-div16 div32}; do
  timeout -k 5 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch $B --n $N --iters ${IT:-10} --tag b${B}_${N}_$V
done
