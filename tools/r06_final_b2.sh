# Round-6 final pass, part b on the final binary: kernel stats, fused-vs-batched PMC and the
# k_compact_mag1 PMC traffic (calibrated) that bench.py's roofline.traffic reads.
set -o pipefail
TAG=${TAG:-r06e} bash tools/r06_final.sh b &&
bash tools/pmc_round.sh ${TAG:-r06e}_pmcround > gpurun_out/${TAG:-r06e}_pmcround.log 2>&1 &&
tail -3 gpurun_out/${TAG:-r06e}_pmcround.log
