# A/B of sample segments per workgroup (one process each): single 128 M gradient, 64-client batch.
set -e
timeout -k 10 120 python tools/kbench.py --iters 10 --tag single_ss4
for V in ss8 ss16; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --iters 10 --tag single_$V
done
timeout -k 10 120 python tools/kbench.py --batch 64 --iters 3 --tag b64_ss4
for V in ss8 ss16; do
  timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$V.so --batch 64 --iters 3 --tag b64_$V
done
