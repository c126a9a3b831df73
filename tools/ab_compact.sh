# A/B of k_compact_mag1 builds (one process each, 64 clients x 128 M per launch, one stream).
set -e
timeout -k 10 120 python tools/kbench.py --batch 64 --iters 4 --tag il1
for V in il32 il64 il8r il32r il64r; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch 64 --iters 4 --tag $V
done
timeout -k 10 120 python tools/kbench.py --batch 64 --iters 4 --tag il1_again
