set -e
cd /tmp && export TMPDIR=/tmp
cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kb -o kb -- python3 tools/kbench.py --tag prof > gpurun_out/prof_kb.log 2>&1
find gpurun_out/prof_kb -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20
