# rocprofv3 PMC passes over k_fold_q (128 packets of 128 M, tools/kbench.py --dec): SQ cycle
# breakdown + LDS, then HBM bytes.  One counter group per pass, each under a KILL timeout.
#   gpurun --timeout 600 -- 'bash tools/pmc_fold.sh r02_pmc_fold'
set -e
TAG=${1:-pmc_fold}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters
  timeout -s KILL 150 rocprofv3 --pmc $2 -d $OUT/$1 -o p -- python3 tools/kbench.py --dec 128 --iters 1 --tag pmc > $OUT/$1.log 2>&1
  python3 tools/rocpd_summary.py counters $(find $OUT/$1 -name "*.db" | head -1) k_fold_q > $OUT/$1.json
  cat $OUT/$1.json
}
run sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS"
run fetch "FETCH_SIZE"
run ta "TA_BUSY_avr TA_TA_BUSY_sum"
echo "[pmc_fold] done"
