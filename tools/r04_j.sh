# Round-4 pass J: the headline step (128 x 128 M) with the batched encode on 1 vs 2 streams,
# alternating processes.
set -e
OUT=gpurun_out/${1:-r04_j}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for s in 2 1; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-single --no-matrix --steps 100 \
      --streams $s > $OUT/h_s${s}_$i.json
    python -c "import json,sys; d=json.loads(open('$OUT/h_s${s}_$i.json').read().strip().splitlines()[-1]); print('streams', $s, 'rep', $i, d['value'], d['ms_per_step'], d['extra']['configs_1_2']['config2_128x16M']['ms_per_step'] if 'configs_1_2' in d['extra'] else '')"
  done
done
echo "[r04_j] done"
