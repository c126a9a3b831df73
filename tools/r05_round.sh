# Round-5 measurement pass (one GPU call): the GPU suite + smoke + the default bench +
# rocprofv3 kernel stats (the bench's step, the lone dense 128 M encode, configs[1]/[2]) +
# the k_compact_mag1 PMC traffic passes for this binary.
#   gpurun --timeout 1500 -- 'bash tools/r05_round.sh <tag>'
set -e
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_round.sh $TAG
echo "[r05_round] rocprofv3 kernel stats (configs[1] / configs[2])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c12 -o c12 -- \
  python3 tools/c2_probe.py --steps 50 > $OUT/prof_c12.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof_c12 -name "*.db" | head -1) $OUT/kernel_stats_configs12.csv
bash tools/pmc_round.sh ${TAG}_pmc
echo "[r05_round] done"
