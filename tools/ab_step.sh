# A/B of whole bench steps (headline workload) across libfedcodec.so builds in tools/variants/.
set -e
timeout -k 10 200 python bench.py --steps 20 --no-single --no-cpu-baseline --roofline-steps 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': 'default', 'value': d['value'], 'ms': d['ms_per_step'], 'k': d['extra']['per_step_kernel_time']}))"
for V in ${VARS:-seg512 seg256}; do
  timeout -k 10 200 python bench.py --steps 20 --no-single --no-cpu-baseline --roofline-steps 0 --lib tools/variants/lib_$V.so | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$V', 'value': d['value'], 'ms': d['ms_per_step'], 'k': d['extra']['per_step_kernel_time']}))"
done
