# Single-client fused dense encode (16 M, 128 M) for libfedcodec.so builds in tools/variants/.
set -e
for N in 16777216 134217728; do
  timeout -k 5 100 python tools/sample_probe.py --n $N --dense --iters 50 --tag default | grep '^{'
  for V in ${VARS:-sw8 sw16}; do
    timeout -k 5 100 python tools/sample_probe.py --lib tools/variants/lib_$V.so --n $N --dense --iters 50 --tag $V | grep '^{'
  done
done
