# rocprofv3 PMC passes over k_compact_mag1 (128 clients x 128 M per launch, tools/kbench.py
# --batch 128): SQ cycle breakdown + LDS + VALU, then TA.  One counter group per pass.
#   gpurun --timeout 600 -- 'bash tools/pmc_compact.sh r02_pmc_compact'
set -e
TAG=${1:-pmc_compact}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters
  timeout -s KILL 170 rocprofv3 --pmc $2 -d $OUT/$1 -o p -- python3 tools/kbench.py --batch 128 --iters 1 --tag pmc > $OUT/$1.log 2>&1
  python3 tools/rocpd_summary.py counters $(find $OUT/$1 -name "*.db" | head -1) k_compact_mag1 > $OUT/$1.json
  cat $OUT/$1.json
}
run sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS"
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES"
run ta "TA_BUSY_avr TA_TA_BUSY_sum"
echo "[pmc_compact] done"
