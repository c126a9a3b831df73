# Round-6 A/B: batched magnitude encode binning its candidates in k_compact_mag1 (no
# k_resolve<true>): parity subset first, then configs[1]/[2] and the headline step.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_batchbin.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "batch or configs2 or configs3 or host_ring or equals_single" --timeout 300 --timeout-method thread > gpurun_out/r06_batchbin_tests.log 2>&1 &&
tail -3 gpurun_out/r06_batchbin_tests.log &&
git_base=tools/variants/lib_base_r06b.so &&
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_batchbin.jsonl --reps 3 \
  --var base=$git_base --var batchbin=tools/variants/lib_batchbin.so \
  --probe "tools/c2_probe.py --steps 100" --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix" > gpurun_out/r06_ab_batchbin.log 2>&1
