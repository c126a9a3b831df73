# Round-6 final pass on the final binary (two calls, each within the 20-minute limit):
#   part a: GPU suite, smoke, default bench      -> gpurun_out/r06c/
#   part b: rocprofv3 kernel stats + the fused-vs-batched PMC passes
set -o pipefail
PART=${1:-a}
if [ "$PART" = a ]; then
  SKIP_PROF=1 SKIP_PMC=1 bash tools/r06_round.sh ${TAG:-r06c}
else
  SKIP_TESTS=1 SKIP_BENCH=1 SKIP_PMC=1 bash tools/r06_round.sh ${TAG:-r06c} &&
  bash tools/pmc_r06.sh ${TAG:-r06c}_pmc > gpurun_out/${TAG:-r06c}_pmc.log 2>&1
fi
