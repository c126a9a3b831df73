# A/B of sample sizes on the single-gradient path (one process each).
set -e
timeout -k 10 120 python tools/kbench.py --iters 10 --tag single_s1024
for V in s512 s256; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --iters 10 --tag single_$V
done
