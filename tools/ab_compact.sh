# Dense decode grid A/B on the single-gradient path (FC_DECODE_GRID overrides the WG count).
set -e
timeout -k 10 120 python tools/kbench.py --iters 10 --tag grid768
FC_DECODE_GRID=1024 timeout -k 10 120 python tools/kbench.py --iters 10 --tag grid1024
FC_DECODE_GRID=2048 timeout -k 10 120 python tools/kbench.py --iters 10 --tag grid2048
FC_DECODE_GRID=16384 timeout -k 10 120 python tools/kbench.py --iters 10 --tag grid16384
