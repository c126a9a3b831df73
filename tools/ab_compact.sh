set -e
timeout -k 10 120 python tools/kbench.py --batch 32 --iters 5 --tag s1024
timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_s512.so --batch 32 --iters 5 --tag s512
timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_s256.so --batch 32 --iters 5 --tag s256
