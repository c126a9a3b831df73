# A/B of sample histogram shards (one process each): single 128 M gradient, 64-client batch.
set -e
timeout -k 10 120 python tools/kbench.py --iters 10 --tag single_sh8
for V in sh1 sh4 sh16; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --iters 10 --tag single_$V
done
timeout -k 10 120 python tools/kbench.py --batch 64 --iters 3 --tag b64_sh8
for V in sh1 sh4 sh16; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch 64 --iters 3 --tag b64_$V
done
