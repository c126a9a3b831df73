set -e
VARS="seg2048 seg4096 div32" bash tools/ab_single.sh
for V in base4 seg2048 base4 seg2048; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-single --steps 100 --lib tools/variants/lib_$V.so > gpurun_out/b_$V.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'v':sys.argv[2],'value':d['value'],'ms':d['ms_per_step'],'roof':d['roofline']['frac']}))" gpurun_out/b_$V.json $V
done
