# Round-6: k_decode_res with the bin search in its workgroup 0 (no k_beta launch): parity, then
# the same-box A/B against the previous library (tools/variants/lib_base.so).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "encode_decode or concurrent or graph or stall" \
  --timeout 120 --timeout-method thread > gpurun_out/r06_bid2_tests.log 2>&1 &&
tail -3 gpurun_out/r06_bid2_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_bid2.jsonl --reps 4 \
  --var base=tools/variants/lib_base.so --var bid2= \
  --probe "tools/encdec_probe.py --n 134217728" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_bid2.log 2>&1
