# Round-6 A/B: four sample segments per workgroup at every n.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_segs4.jsonl --reps 4 \
  --var base= --var segs4=tools/variants/lib_segs4.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/c2_probe.py --steps 100" > gpurun_out/r06_ab_segs4.log 2>&1
