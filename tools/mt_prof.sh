# rocprofv3 kernel stats of the device MT19937 draws (8 rows of 25.5 M) + the full-size Aggregator rates
set -e
OUT=gpurun_out/${1:-mtprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o mt -- python3 tools/mt_gpu_check.py > $OUT/prof.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof -name "*.db" | head -1) $OUT/kernel_stats_mt.csv
grep -i "mt_" $OUT/kernel_stats_mt.csv | cut -d, -f1-6
timeout -k 10 600 python -u -m pytest "tests/test_fullsize_parity.py::test_configs4_device_aggregator_other_codecs" \
  -x -q -s --timeout 300 --timeout-method thread -k "dropout" > $OUT/fullsize.log 2>&1 || { tail -40 $OUT/fullsize.log; exit 1; }
grep "GB/s" $OUT/fullsize.log
