# Quick A/B pass of the default build: GPU parity tests, then kernel timings of the batched
# encode (16 M x 64, 128 M x 8) and the single-gradient dense path (16 M, 128 M).
set -e
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
fi
timeout -k 5 120 python tools/kbench.py --batch 64 --n 16777216 --iters 10 --tag b64_16M
timeout -k 5 120 python tools/kbench.py --batch 8 --n 134217728 --iters 10 --tag b8_128M
for N in 16777216 134217728; do
  timeout -k 5 100 python tools/sample_probe.py --n $N --dense --iters 50 --tag dense | grep '^{'
done
