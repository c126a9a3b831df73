# Round-6 A/B (timing only): the price of the library's per-call ordering event.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_noguard.jsonl --reps 4 \
  --var base= --var noguard=tools/variants/lib_noguard.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_noguard.log 2>&1
