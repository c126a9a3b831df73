set -e
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 120 python tools/kbench.py --batch 16 --iters 5 --tag mag1
FC_MAG_KERNEL=2 FC_MAG_GRID=768 timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_w6.so --batch 16 --iters 5 --tag pers_w6_768
FC_MAG_KERNEL=2 FC_MAG_GRID=512 timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_w4.so --batch 16 --iters 5 --tag pers_w4_512
FC_MAG_KERNEL=2 FC_MAG_GRID=1024 timeout -k 10 120 python tools/kbench.py --lib tools/variants/lib_w4.so --batch 16 --iters 5 --tag pers_w4_1024
timeout -k 10 120 python tools/kbench.py --iters 5 --tag single
