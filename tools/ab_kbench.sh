# Same-box A/B of library builds on tools/kbench.py probes, alternating (two rounds).
#   gpurun -- 'bash tools/ab_kbench.sh <out.jsonl> "<probe args>" <tag>=<lib.so> <tag>=<lib.so> ...'
set -e
OUT=$1; PROBE=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for r in 1 2; do
  for v in "$@"; do
    timeout -k 10 240 python -u tools/kbench.py $PROBE --lib "${v#*=}" --tag "${v%%=*}" | tail -1 | tee -a "$OUT"
  done
done
