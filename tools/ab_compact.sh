set -e
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 120 python tools/kbench.py --batch 16 --iters 5 --tag wave6
timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_w8.so --batch 16 --iters 5 --tag wave8
FC_COMPACT=mag1 timeout -k 10 120 python tools/kbench.py --batch 16 --iters 5 --tag mag1
