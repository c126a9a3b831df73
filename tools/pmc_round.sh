# rocprofv3 PMC passes for roofline.traffic (one counter group per pass, each under its own
# KILL timeout; MI355X_MICROARCH.md §HBM + the rocprofv3 PMC rules):
#   1. calibration: known 512 MiB dispatches in k_compact_mag1's access shapes (FETCH, WRITE)
#   2. k_compact_mag1 at 128 clients x 134,217,728 per launch (FETCH, WRITE)
#   gpurun --timeout 900 -- 'bash tools/pmc_round.sh r02_pmc'
set -e
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
N=134217728
K=13421773
echo "[pmc] calibration"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cal_f -o cal -- python3 tools/pmc_calib.py > $OUT/cal_f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/cal_w -o cal -- python3 tools/pmc_calib.py > $OUT/cal_w.log 2>&1
python3 tools/rocpd_summary.py calib $(find $OUT/cal_f -name "*.db" | head -1) \
  $(find $OUT/cal_w -name "*.db" | head -1) $OUT/pmc_calib.json
echo "[pmc] k_compact_mag1, 128 clients per launch"
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_f -o pmc -- python3 tools/kbench.py --batch 128 --iters 2 --tag pmc > $OUT/pmc_f.log 2>&1
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_w -o pmc -- python3 tools/kbench.py --batch 128 --iters 2 --tag pmc > $OUT/pmc_w.log 2>&1
python3 tools/rocpd_summary.py pmc $(find $OUT/pmc_f -name "*.db" | head -1) \
  $(find $OUT/pmc_w -name "*.db" | head -1) k_compact_mag1 $OUT/pmc_k_compact_mag1.json \
  --alg-bytes $((128 * (4 * N + 8 * K))) --clients-per-launch 128 --calib $OUT/pmc_calib.json
echo "[pmc] done"
