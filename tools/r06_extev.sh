# Round-6: the fused launches carry the library's ordering event themselves
# (hipExtLaunchKernelGGL stop event) instead of a hipEventRecord packet after them.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_f64_boundary.py -m gpu -x -q \
  -k "concurrent or ordered or stall or graph or encode_decode or fused or f64" --timeout 200 --timeout-method thread > gpurun_out/r06_extev_tests.log 2>&1 &&
tail -2 gpurun_out/r06_extev_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_extev.jsonl --reps 4 \
  --var base=tools/variants/lib_srec_adopted.so --var extev= \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_extev.log 2>&1
