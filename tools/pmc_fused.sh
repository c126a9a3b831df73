# rocprofv3 PMC passes over the lone-client fused encode (k_fused_mag<false> packet vs
# k_fused_mag<true> dense, one 128 M gradient, tools/fused_probe.py).  One counter group per
# pass, each under its own KILL timeout.
#   gpurun --timeout 600 -- 'bash tools/pmc_fused.sh r04_pmc_fused'
set -e
TAG=${1:-pmc_fused}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, mode, counters
  timeout -s KILL 90 rocprofv3 --pmc $3 -d $OUT/$1_$2 -o p -- python3 tools/fused_probe.py --mode $2 > $OUT/$1_$2.log 2>&1
  python3 tools/rocpd_summary.py counters $(find $OUT/$1_$2 -name "*.db" | head -1) k_fused_mag > $OUT/$1_$2.json
  echo "== $1 $2"; cat $OUT/$1_$2.json
}
for m in packet dense; do
  run fetch $m "FETCH_SIZE"
  run write $m "WRITE_SIZE"
  run sq $m "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
  run sq2 $m "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
done
echo "[pmc_fused] done"
