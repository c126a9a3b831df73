# Round-6 A/B (timing): the batched compaction computing each client's gradient pointer from a
# slab hint instead of loading it from the job table ahead of its gradient loads.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python tools/ab.py --out gpurun_out/r06_ab_slabhint.jsonl --reps 3 \
  --var base= --var slabhint=tools/variants/lib_slabhint.so \
  --probe "tools/c2_probe.py --steps 100" --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix" > gpurun_out/r06_ab_slabhint.log 2>&1
