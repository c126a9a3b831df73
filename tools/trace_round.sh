# Phase traces of the small encode kernels for the FC_TRACE builds in tools/variants/.
set -e
for V in ${VARS:-trace trace_plain trace_nopilot}; do
  for N in ${NS:-134217728 16777216}; do
    timeout -k 5 100 python tools/trace_probe.py --lib tools/variants/lib_$V.so --n $N --dense | sed "s/^{/{\"v\": \"$V\", /"
  done
done
