set -e
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
FC_COMPACT=mag4 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "top or batch or fedavg" --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1 || { tail -40 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
timeout -k 10 120 python tools/kbench.py --batch 16 --iters 5 --tag mag1
FC_COMPACT=mag4 timeout -k 10 120 python tools/kbench.py --batch 16 --iters 5 --tag mag4_w6
FC_COMPACT=mag4 timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_m4w5.so --batch 16 --iters 5 --tag mag4_w5
FC_COMPACT=mag4 timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_m4w4.so --batch 16 --iters 5 --tag mag4_w4
