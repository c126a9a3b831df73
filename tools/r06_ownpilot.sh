# Round-6 A/B: k_fused_mag's sample workgroups computing the pilot window themselves (always /
# only for two-segment pilots, n <= 32 M).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_ownpilot2.jsonl --reps 6 \
  --var base= --var ownpilot=tools/variants/lib_ownpilot.so --var ownsmall=tools/variants/lib_ownsmall.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_ownpilot2.log 2>&1
