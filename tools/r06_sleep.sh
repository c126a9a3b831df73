# Round-6 A/B: k_fused_mag's first-round start delay (s_sleep 90 -> 45 / 140) after the own-pilot
# and scalar-record changes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_sleep.jsonl --reps 4 \
  --var base= --var sleep45=tools/variants/lib_sleep45.so --var sleep140=tools/variants/lib_sleep140.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_sleep.log 2>&1
