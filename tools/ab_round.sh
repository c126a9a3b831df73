set -e
bash tools/gpu_ab.sh dual
N=16777216 B=64 VARS="rgb32 rgb64" bash tools/ab_batch16.sh
N=134217728 B=16 IT=6 VARS="rgb32 rgb64" bash tools/ab_batch16.sh
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/dual_bench.json 2> gpurun_out/dual_bench.err
python3 -c "
import json; d=json.load(open('gpurun_out/dual_bench.json')); e=d['extra']
print(json.dumps({'value':d['value'],'ms':d['ms_per_step'],'roof':d['roofline']['frac'],'k':{c:v['avg_us'] for c,v in e['per_step_kernel_time'].items() if c!='note'},'single':e['single_gradient']['fused_dense'],'c1':e['configs_1_2']['config1_single_16M']['fused_dense'],'c2':e['configs_1_2']['config2_128x16M']['hbm_frac'], 'c2ms':e['configs_1_2']['config2_128x16M']['ms_per_step'],'self':e['self_check'][:3]}))"
