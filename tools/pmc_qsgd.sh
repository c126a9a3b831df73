# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) for the QSGD kernels: one 128 M 2-bit encode +
# decode and a fold of 70 x 25,557,032 2-bit packets (tools/qsgd_probe.py), each pass under its
# own KILL timeout.   gpurun --timeout 600 -- 'bash tools/pmc_qsgd.sh r05_pmc_qsgd'
set -e
TAG=${1:-pmc_qsgd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
N=134217728
NF=25557032
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o p -- python3 tools/qsgd_probe.py --iters 3 --fold 70 > $OUT/f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o p -- python3 tools/qsgd_probe.py --iters 3 --fold 70 > $OUT/w.log 2>&1
F=$(find $OUT/f -name "*.db" | head -1); W=$(find $OUT/w -name "*.db" | head -1)
python3 tools/rocpd_summary.py pmc $F $W k_qsgd_norm $OUT/norm.json --alg-bytes $((4 * N))
python3 tools/rocpd_summary.py pmc $F $W k_qsgd_quant $OUT/quant.json --alg-bytes $((4 * N + N / 2))
python3 tools/rocpd_summary.py pmc $F $W "k_qsgd_decode<false>" $OUT/decode.json --alg-bytes $((4 * N + N / 2))
python3 tools/rocpd_summary.py pmc $F $W "k_qsgd_decode<true>" $OUT/fold.json --alg-bytes $((70 * NF / 2 + 4 * NF))
echo "[pmc_qsgd] done"
