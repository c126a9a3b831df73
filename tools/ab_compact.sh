# A/B of the sample size cap on 64-client batches of 16 M gradients (one process each).
set -e
timeout -k 10 120 python tools/kbench.py --n 16777216 --batch 64 --iters 5 --tag s512
for V in s256 s128; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --n 16777216 --batch 64 --iters 5 --tag $V
done
