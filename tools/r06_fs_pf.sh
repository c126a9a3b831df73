# Round-6: full-size Aggregator rates (device MT dropout) + the bracket-wait prefetch A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_fullsize_parity.py::test_configs4_device_aggregator_other_codecs" \
  -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r06_fullsize_agg.log 2>&1 &&
grep -E "GB/s|passed|failed" gpurun_out/r06_fullsize_agg.log &&
timeout -k 10 400 python -u tools/mt_agg_probe.py > gpurun_out/r06_mt_agg_probe.log 2>&1 &&
grep -v amdgpu.ids gpurun_out/r06_mt_agg_probe.log | tail -8 &&
timeout -k 10 900 python tools/ab.py --out gpurun_out/r06_ab_prefetch.jsonl --reps 3 \
  --var base= --var pf1=tools/variants/lib_pf1.so --var pf2=tools/variants/lib_pf2.so --var pf4=tools/variants/lib_pf4.so \
  --probe "tools/encdec_probe.py --n 134217728" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_prefetch.log 2>&1
