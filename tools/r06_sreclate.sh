# Round-6 A/B: the scalar bracket record loaded after the gradient loads, dense form included.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_sreclate.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or single_client or dense or concurrent" --timeout 300 --timeout-method thread > gpurun_out/r06_sreclate_tests.log 2>&1 &&
tail -2 gpurun_out/r06_sreclate_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_sreclate.jsonl --reps 5 \
  --var base=tools/variants/lib_decpro.so --var sreclate=tools/variants/lib_sreclate.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_sreclate.log 2>&1
