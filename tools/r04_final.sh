# Round-4 final pass: GPU suite + smoke + bench + kernel stats (tools/gpu_round.sh), then the
# k_compact_mag1 PMC passes for the shipped binary (tools/pmc_round.sh).
set -e
bash tools/gpu_round.sh ${1:-r04_final}
bash tools/pmc_round.sh ${1:-r04_final}_pmc
echo "[r04_final] done"
