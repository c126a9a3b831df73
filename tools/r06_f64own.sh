# Round-6 A/B: k_fused64's sample workgroups computing the pilot window themselves.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab.py --out gpurun_out/r06_ab_f64own.jsonl --reps 4 \
  --var base= --var f64own=tools/variants/lib_f64own.so \
  --probe "tools/f64top_probe.py --n 16777216" --probe "tools/f64top_probe.py --n 67108864" > gpurun_out/r06_ab_f64own.log 2>&1
