# Round-4 pass N: does the headline run before it slow bench.small_configs (configs[2])?
# Full headline (300 steps) vs a 3-step headline, alternating; then c2_diag alone.
set -e
OUT=gpurun_out/r04_n
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for s in 300 3; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matrix --steps $s > $OUT/b_${s}_$i.json
    python -c "import json; d=json.loads(open('$OUT/b_${s}_$i.json').read().strip().splitlines()[-1]); c=d['extra']['configs_1_2']; print('steps', $s, 'rep', $i, d['ms_per_step'], c['config2_128x16M']['ms_per_step'], c['config1_single_16M']['fused_dense']['us'])"
  done
done
timeout -k 10 120 python -u tools/c2_diag.py --reps 2 --steps 100 --modes top1
echo "[r04_n] done"
