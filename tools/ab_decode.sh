# A/B of k_decode_sparse<true> builds over 128 distinct 128 M-float top-k packets (one process each).
set -e
for V in b64 occ4 occ3n b64; do
  timeout -k 10 180 python tools/kbench.py --lib tools/variants/lib_$V.so --dec 128 --iters 5 --tag $V
done
