set -e
for r in 1 2 3; do
  timeout -k 10 200 python tools/c2_probe.py --steps 100 --tag slab
  timeout -k 10 200 python tools/c2_probe.py --steps 100 --separate-packets --tag sep
done
