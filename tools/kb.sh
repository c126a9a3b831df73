set -e
cd /root/repo
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python tools/kbench.py --tag main
for t in ${VARIANTS:-}; do timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_$t.so --tag $t; done
