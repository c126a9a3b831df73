# Whole-step bench A/B of libfedcodec.so variants (tools/variants/lib_<V>.so), two passes.
set -e
for P in 1 2; do
for V in ${VARS:-cur}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single --steps ${STEPS:-100} --lib tools/variants/lib_$V.so > gpurun_out/b_$V.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['extra']['per_step_kernel_time']; print(json.dumps({'v':sys.argv[2],'value':d['value'],'ms':d['ms_per_step'],'roof':d['roofline']['frac'],'sample':k['sample']['avg_us'],'engine':k['engine']['avg_us'],'compact':k['compact']['avg_us']}))" gpurun_out/b_$V.json $V
done
done
