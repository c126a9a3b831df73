# A/B of k_compact_mag1 builds (one process each, 128 clients x 128 M per launch, one stream).
set -e
timeout -k 10 120 python tools/kbench.py --batch 128 --iters 3 --tag il64
for V in plain il128 w6; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch 128 --iters 3 --tag $V
done
