# Round-4 A/B + trace pass (one gpurun call):
#   gpurun --timeout 1190 -- 'bash tools/r04_ab.sh r04_ab'
# 1. sample chain: pilot-first gate x 64-bit flush (lone packet / dense, 128 M and 16 M; batched 64 x 16 M)
# 2. QSGD: reverse-order quantise, plain loads
# 3. FC_TRACE phase timelines (gate+flush64 vs neither)
# 4. configs[4] end-to-end at 1 GPU, ring vs sequential
set -e
TAG=${1:-r04_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python tools/ab.py --out $OUT/ab_sample.jsonl --reps 2 --timeout 100 \
  --var g1f1= --var g0f0=tools/variants/lib_g0f0.so --var g1f0=tools/variants/lib_g1f0.so \
  --var g0f1=tools/variants/lib_g0f1.so \
  --probe "tools/sample_probe.py --n 134217728" --probe "tools/sample_probe.py --n 134217728 --dense" \
  --probe "tools/sample_probe.py --n 16777216 --dense" --probe "tools/sample_probe.py --n 16777216" \
  --probe "tools/kbench.py --batch 64 --n 16777216"
timeout -k 10 200 python tools/ab.py --out $OUT/ab_qsgd.jsonl --reps 2 --timeout 100 \
  --var new= --var r0=tools/variants/lib_qsgd_r0.so --var r0p0=tools/variants/lib_qsgd_r0p0.so \
  --probe "tools/qsgd_probe.py --n 134217728"
for V in trace trace_g0f0; do
  for a in "--n 134217728 --dense" "--n 134217728" "--n 16777216 --dense"; do
    timeout -k 5 100 python tools/trace_probe.py --lib tools/variants/lib_$V.so $a | sed "s/^{/{\"v\": \"$V\", /" >> $OUT/traces.jsonl
  done
done
timeout -k 10 250 python -u tools/e2e_bench.py --mode ring > $OUT/e2e_ring.json 2> $OUT/e2e_ring.err
timeout -k 10 250 python -u tools/e2e_bench.py --mode reduce > $OUT/e2e_seq.json 2> $OUT/e2e_seq.err
cat $OUT/e2e_ring.json $OUT/e2e_seq.json
echo "[r04_ab] done"
