# Round-6 A/B: k_fused64 later chunk workgroups reading the bracket record with a scalar load.
set -o pipefail
mkdir -p gpurun_out
cp tools/variants/lib_f64srec.so openmsftl_amd/libfedcodec.so &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_f64_boundary.py -m gpu -x -q -k "f64 or fp64 or float64" \
  --timeout 200 --timeout-method thread > gpurun_out/r06_f64srec_tests.log 2>&1 &&
tail -2 gpurun_out/r06_f64srec_tests.log &&
timeout -k 10 600 python tools/ab.py --out gpurun_out/r06_ab_f64srec.jsonl --reps 4 \
  --var base=tools/variants/lib_srec_adopted.so --var f64srec=tools/variants/lib_f64srec.so \
  --probe "tools/f64top_probe.py --n 16777216" --probe "tools/f64top_probe.py --n 67108864" > gpurun_out/r06_ab_f64srec.log 2>&1
