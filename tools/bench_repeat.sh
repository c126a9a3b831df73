# The default bench three times back to back on one box (run-to-run spread of the final tree).
set -e
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/rep_$i.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']; c=e['configs_1_2']; print(json.dumps({'run':int(sys.argv[2]),'value':d['value'],'ms':d['ms_per_step'],'roofline_frac':d['roofline']['frac'],'step_frac':e['step_roofline']['frac'],'single128M_dense':e['single_gradient']['fused_dense'],'configs1_dense':c['config1_single_16M']['fused_dense'],'configs2_frac':c['config2_128x16M']['hbm_frac'],'configs2_ms':c['config2_128x16M']['ms_per_step'],'fold_us':e['per_step_kernel_time']['decode']['avg_us']}))" gpurun_out/rep_$i.json $i
done
