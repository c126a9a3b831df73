# Round-6 A/B: later-round chunk workgroups of k_fused_mag reading the bracket record with a
# scalar load issued before their gradient loads (FC_FUSED_SREC = first chunk that tries it).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python tools/ab.py --out gpurun_out/r06_ab_srec.jsonl --reps 4 \
  --var base= --var srec1k=tools/variants/lib_srec1k.so --var srec2k=tools/variants/lib_srec2k.so \
  --var srec4k=tools/variants/lib_srec4k.so \
  --probe "tools/encdec_probe.py --n 134217728" --probe "tools/encdec_probe.py --n 16777216" > gpurun_out/r06_ab_srec.log 2>&1
