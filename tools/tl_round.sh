set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl/cfg2 -o cfg2 -- python3 bench.py --n 16777216 --steps 6 --warmup 2 --no-single --no-cpu-baseline --roofline-steps 0 > gpurun_out/tl/cfg2.log 2>&1
python3 tools/rocpd_summary.py timeline $(find gpurun_out/tl/cfg2 -name "*.db" | head -1) 40 > gpurun_out/tl/cfg2_timeline.txt
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl/c3 -o c3 -- python3 bench.py --steps 4 --warmup 2 --no-single --no-cpu-baseline --roofline-steps 0 > gpurun_out/tl/c3.log 2>&1
python3 tools/rocpd_summary.py timeline $(find gpurun_out/tl/c3 -name "*.db" | head -1) 30 > gpurun_out/tl/c3_timeline.txt
