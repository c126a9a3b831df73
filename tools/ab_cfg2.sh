# A/B of BASELINE configs[2] (128 clients x 16 M: batched encode on two streams + fold) across
# libfedcodec.so builds in tools/variants/ (bench.py's main loop at n = 16 M).
set -e
one() {  # tag, extra args
  timeout -k 10 200 python bench.py --n 16777216 --steps 40 --no-single --no-cpu-baseline --roofline-steps 0 $2 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$1', 'value': d['value'], 'ms': d['ms_per_step'], 'k': d['extra']['per_step_kernel_time']}))"
}
one default ""
for V in ${VARS:-div128 rgb16 rgb32}; do one $V "--lib tools/variants/lib_$V.so"; done
