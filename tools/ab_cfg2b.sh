# configs[2]-shaped step (128 clients x 16 M, encode + fold, bench.py main loop) per variant.
set -e
for P in 1 2; do
for V in ${VARS:-cur}; do
  timeout -k 10 300 python -u bench.py --n 16777216 --no-cpu-baseline --no-single --steps 200 --roofline-steps 0 --lib tools/variants/lib_$V.so > gpurun_out/c2_$V.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['extra']['per_step_kernel_time']; print(json.dumps({'v':sys.argv[2],'value':d['value'],'ms':d['ms_per_step'],'step_frac':d['extra']['step_roofline']['frac'],'sample':k['sample']['avg_us'],'engine':k['engine']['avg_us'],'compact':k['compact']['avg_us'],'fallbacks':d['extra']['exact_fallbacks']}))" gpurun_out/c2_$V.json $V
done
done
