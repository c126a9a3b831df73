# A/B of the encode's small launches: diagnostic ablation builds of k_sample1 / k_resolve
# (tools/variants/lib_{s,r}N.so), one process each, dense single-gradient path.
set -e
VARS=${VARS:-"s1 s2 s3 s4 r1 r2 r3 r4 r5"}
for N in ${NS:-134217728 16777216}; do
  timeout -k 10 120 python tools/sample_probe.py --n $N --dense --tag base
  for V in $VARS; do
    timeout -k 10 120 python tools/sample_probe.py --lib tools/variants/lib_$V.so --n $N --dense --tag $V
  done
done
