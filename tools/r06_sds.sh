# Round-6 A/B: the drop-in dense encode's sample size (FC_SAMPLE_DIV_SINGLE 32 -> 16 / 64).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r06_ab_sds.jsonl --reps 4 \
  --var base= --var sds64=tools/variants/lib_sds64.so --var sds16=tools/variants/lib_sds16.so \
  --probe "tools/encdec_probe.py --n 16777216" --probe "tools/encdec_probe.py --n 134217728" > gpurun_out/r06_ab_sds.log 2>&1
