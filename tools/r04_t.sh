# Round-4 pass T: non-temporal packet stores in the batched compaction — headline bench
# (with configs[1]/[2] and the single gradient) against the previous library, alternating;
# then the GPU suite.
set -e
OUT=gpurun_out/r04_t
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in head new; do
    L=""; [ $v = head ] && L="--lib tools/variants/lib_head.so"
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-matrix --steps 100 $L > $OUT/b_${v}_$i.json
    python -c "import json; d=json.loads(open('$OUT/b_${v}_$i.json').read().strip().splitlines()[-1]); e=d['extra']; c=e['configs_1_2']; print(json.dumps({'var': '$v', 'rep': $i, 'value': d['value'], 'ms': d['ms_per_step'], 'compact_us': d['roofline']['avg_launch_us'], 'frac': d['roofline']['frac'], 'k': e['per_step_kernel_time'], 'c2_ms': c['config2_128x16M']['ms_per_step'], 'c2_frac': c['config2_128x16M']['hbm_frac'], 'c1_dense_us': c['config1_single_16M']['fused_dense']['us'], 'single_us': e['single_gradient']['us_per_encode_decode']}))" | tee -a $OUT/ab.jsonl
  done
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo "[r04_t] done"
