# Round-6: the scalar bracket-record read adopted for k_fused_mag<false>: parity subset, then a
# same-box A/B against the r06b library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or fused or concurrent or stall or single_client or encode_top or graph" --timeout 300 --timeout-method thread > gpurun_out/r06_srec2_tests.log 2>&1 &&
tail -2 gpurun_out/r06_srec2_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_srec2.jsonl --reps 4 \
  --var base=tools/variants/lib_base_r06b.so --var srec= \
  --probe "tools/encdec_probe.py --n 134217728" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_srec2.log 2>&1
