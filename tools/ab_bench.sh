# bench.py A/B in one GPU call (boxes differ by 2-4 %): each variant twice, alternating order.
#   gpurun -- 'bash tools/ab_bench.sh <out.jsonl> "<tag>:<bench args>" "<tag>:<bench args>" ...'
set -e
OUT=$1; shift
mkdir -p "$(dirname "$OUT")"
run() {
  local tag=${1%%:*} args=${1#*:}
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-single --no-matrix $args > /tmp/ab_bench.json 2>/dev/null
  python3 -c "
import json,sys; d=json.load(open('/tmp/ab_bench.json')); e=d['extra']
print(json.dumps({'tag':sys.argv[1],'args':sys.argv[2],'value':d['value'],'ms_per_step':d['ms_per_step'],
 'roof':d['roofline']['frac'],'kernels':{c:v['avg_us'] for c,v in e['per_step_kernel_time'].items() if c!='note'}}))" "$tag" "$args" | tee -a "$OUT"
}
for v in "$@"; do run "$v"; done
for ((i=$#; i>=1; i--)); do run "${!i}"; done
