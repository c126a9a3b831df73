# Round-6 final pass, part 2: the strengthened Philox parity test, then the rocprofv3 kernel stats
# of the final binary (bench step, lone round trips, configs[1]/[2], rand-k).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "philox" \
  --timeout 200 --timeout-method thread > gpurun_out/r06_philox_tests.log 2>&1 &&
tail -2 gpurun_out/r06_philox_tests.log &&
SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PMC=1 bash tools/r06_round.sh r06b
