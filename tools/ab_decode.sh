# A/B of k_decode_sparse<true> builds over 128 distinct 128 M-float top-k packets (one process each).
set -e
timeout -k 10 180 python tools/kbench.py --dec 128 --iters 5 --tag base
timeout -k 10 180 python tools/kbench.py --lib tools/variants/lib_nt.so --dec 128 --iters 5 --tag nt
timeout -k 10 180 python tools/kbench.py --dec 128 --iters 5 --tag base_again
