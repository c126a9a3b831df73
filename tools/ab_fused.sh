# A/B of the single-client encode: k_fused_mag (default) against the two-launch form.
set -e
mkdir -p gpurun_out/fused
for N in 16777216 134217728; do
  for U in 0 1; do
    FC_UNFUSED=$U timeout -k 5 100 python tools/sample_probe.py --n $N --dense --iters 50 --tag "unfused$U" | grep '^{'
    FC_UNFUSED=$U timeout -k 5 100 python tools/sample_probe.py --n $N --iters 50 --tag "unfused$U" | grep '^{'
  done
done
