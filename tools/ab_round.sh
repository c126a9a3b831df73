# One A/B box pass: GPU parity tests, single-gradient variants (VARS), then the bench with and
# without the pipelined encode+fold (configs[2] and the headline step).
set -e
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
fi
[ -n "$VARS" ] && bash tools/ab_single.sh
summ() {
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); e=d['extra']
print(json.dumps({'tag':sys.argv[2],'value':d['value'],'ms':d['ms_per_step'],'roof':d['roofline']['frac'],'k':{c:v['avg_us'] for c,v in e['per_step_kernel_time'].items() if c!='note'},'single':e.get('single_gradient',{}).get('fused_dense'),'c1':e.get('configs_1_2',{}).get('config1_single_16M',{}).get('fused_dense'),'c2':e.get('configs_1_2',{}).get('config2_128x16M',{}).get('hbm_frac'),'c2ms':e.get('configs_1_2',{}).get('config2_128x16M',{}).get('ms_per_step'),'self':e['self_check'][:3]}))" $1 $2
}
for B in $BENCH; do
  case $B in
    pipe) A="" ;;
    nopipe) A="--no-pipeline" ;;
  esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 150 $A > $OUT/bench_$B.json 2> $OUT/bench_$B.err
  summ $OUT/bench_$B.json $B
done
