# Round-6 A/B: the candidate loop skipping groups with no candidate.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_candskip.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or single_client or dense or batch or configs2" --timeout 300 --timeout-method thread > gpurun_out/r06_candskip_tests.log 2>&1 &&
tail -2 gpurun_out/r06_candskip_tests.log &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_candskip.jsonl --reps 4 \
  --var base=tools/variants/lib_final.so --var candskip=tools/variants/lib_candskip.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" \
  --probe "tools/c2_probe.py --steps 100" > gpurun_out/r06_ab_candskip.log 2>&1
