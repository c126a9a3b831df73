# Round-6 A/B: chunks per k_resolve workgroup for lone encodes (dense q, packet, rand-k).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_cpw.jsonl --reps 4 \
  --var base= --var cpw16=tools/variants/lib_cpw16.so --var cpw32=tools/variants/lib_cpw32.so --var cpw64=tools/variants/lib_cpw64.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/randk_probe.py --n 16777216" > gpurun_out/r06_ab_cpw.log 2>&1
