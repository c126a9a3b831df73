# Round-6 A/B: one readlane per pair of groups in the staged phase 2.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_rlpair.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q \
  -k "encode_decode or single_client or dense or batch or configs2 or configs3" --timeout 300 --timeout-method thread > gpurun_out/r06_rlpair_tests.log 2>&1 &&
tail -2 gpurun_out/r06_rlpair_tests.log &&
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_rlpair.jsonl --reps 3 \
  --var base=tools/variants/lib_final.so --var rlpair=tools/variants/lib_rlpair.so \
  --probe "tools/c2_probe.py --steps 100" --probe "tools/encdec_probe.py --n 134217728" \
  --probe "bench.py --steps 40 --no-cpu-baseline --no-single --no-matrix" > gpurun_out/r06_ab_rlpair.log 2>&1
