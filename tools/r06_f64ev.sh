# Round-6 A/B: fp64 sampled top-k with the ordering event on k_fused64's own launch (extev) vs
# the separate record (srec_adopted build).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab.py --out gpurun_out/r06_ab_f64ev.jsonl --reps 4 \
  --var base=tools/variants/lib_srec_adopted.so --var extev= \
  --probe "tools/f64top_probe.py --n 16777216" > gpurun_out/r06_ab_f64ev.log 2>&1 &&
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PMC=1 bash tools/r06_round.sh r06c
