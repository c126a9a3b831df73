# Round-6: k_decode_res loads its quarter offsets with the state and drops its first barrier.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or single_client or graph or concurrent" --timeout 300 --timeout-method thread > gpurun_out/r06_decpro_tests.log 2>&1 &&
tail -2 gpurun_out/r06_decpro_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_decpro.jsonl --reps 5 \
  --var base=tools/variants/lib_extev.so --var decpro= \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_decpro.log 2>&1
