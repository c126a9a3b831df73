set -e
OUT=gpurun_out/${1:-lone}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/lone_probe.py > $OUT/lone.jsonl 2>$OUT/lone.err
cat $OUT/lone.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lone -- python3 tools/lone_probe.py > $OUT/prof.log 2>&1
python3 tools/rocpd_summary.py stats $(find $OUT/prof -name "*.db" | head -1) $OUT/kernel_stats_lone.csv
cut -d, -f1-5 $OUT/kernel_stats_lone.csv | head -30
