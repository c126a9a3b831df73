# Round-6: configs[2] and the headline step with the batched encode split over forked streams
# (sub-batches' small kernels beside each other's compaction) and the pipelined encode+fold.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python tools/ab.py --out gpurun_out/r06_ab_c2streams.jsonl --reps 3 --var cur= \
  --probe "tools/c2_probe.py --steps 100" --probe "tools/c2_probe.py --steps 100 --streams 2" \
  --probe "tools/c2_probe.py --steps 100 --streams 2 --pipeline" --probe "tools/c2_probe.py --steps 100 --streams 4 --pipeline" \
  --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix" \
  --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix --streams 2 --pipeline" > gpurun_out/r06_ab_c2streams.log 2>&1
