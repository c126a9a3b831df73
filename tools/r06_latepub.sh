# Round-6 A/B: k_fused_mag's chunk workgroups reading fz_seq after their gradient loads issue.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_latepub.jsonl --reps 5 \
  --var base= --var latepub=tools/variants/lib_latepub.so \
  --probe "tools/encdec_probe.py --n 134217728" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_latepub.log 2>&1
