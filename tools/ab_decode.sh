# Fold grid A/B over 128 distinct 128 M-float top-k packets (FC_DECODE_GRID overrides the WG count).
set -e
timeout -k 10 180 python tools/kbench.py --dec 128 --iters 5 --tag g768
for G in 1536 4096 16384; do
  FC_DECODE_GRID=$G timeout -k 10 180 python tools/kbench.py --dec 128 --iters 5 --tag g$G
done
