# Round-4 pass AM: the default bench three times on one box (spread of value, configs[1]/[2],
# the single gradient) for the final library.
set -e
OUT=gpurun_out/r04_am
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/b_$i.json
  python -c "import json; d=json.loads(open('$OUT/b_$i.json').read().strip().splitlines()[-1]); e=d['extra']; c=e['configs_1_2']; print(json.dumps({'rep': $i, 'value': d['value'], 'ms': d['ms_per_step'], 'frac': d['roofline']['frac'], 'c2_ms': c['config2_128x16M']['ms_per_step'], 'c2_frac': c['config2_128x16M']['hbm_frac'], 'c1_dense_us': c['config1_single_16M']['fused_dense']['us'], 'c1_frac': c['config1_single_16M']['fused_dense']['hbm_frac'], 'single_us': e['single_gradient']['us_per_encode_decode'], 'single_frac': e['single_gradient']['hbm_frac'], 'dense_us': e['single_gradient']['fused_dense']['us'], 'dense_frac': e['single_gradient']['fused_dense']['hbm_frac'], 'qsgd_frac': e['qsgd_single_gradient']['hbm_frac'], 'fp64_frac': e['codec_matrix']['top_f0.1_16M_fp64']['hbm_frac']}))" | tee -a $OUT/summary.jsonl
done
echo "[r04_am] done"
