# A/B of k_fold_q tilings (FC_QR entry rounds x FC_QG items per group) on 128 distinct
# 128 M packets (tools/kbench.py --dec), one process per build.
set -e
timeout -k 10 200 python tools/kbench.py --dec 128 --iters 3 --tag default
for V in ${VARS:-qr5g4 qr5g2}; do
  timeout -k 10 200 python tools/kbench.py --lib tools/variants/lib_$V.so --dec 128 --iters 3 --tag $V
done
