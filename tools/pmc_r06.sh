# Round-6 PMC passes: the lone fused packet encode (k_fused_mag<false>, via fc_topk_encode_decode)
# against the batched compaction of the same gradient (k_compact_mag1, one client), 128 M.
set -e
TAG=${1:-r06_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, mode, kernel, counters
  timeout -s KILL 90 rocprofv3 --pmc $4 -d $OUT/$1_$2 -o p -- python3 tools/fused_probe.py --mode $2 > $OUT/$1_$2.log 2>&1
  python3 tools/rocpd_summary.py counters $(find $OUT/$1_$2 -name "*.db" | head -1) $3 > $OUT/$1_$2.json
  echo "== $1 $2"; cat $OUT/$1_$2.json
}
for m in encdec:k_fused_mag batch1:k_compact_mag1; do
  mode=${m%%:*}; kern=${m##*:}
  run sq $mode $kern "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"
  run sq2 $mode $kern "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
done
run fetch encdec k_decode_res "FETCH_SIZE"
run write encdec k_decode_res "WRITE_SIZE"
echo "[pmc_r06] done"
