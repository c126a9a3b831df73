set -e
VARS="ss4 ss16 cur" bash tools/ab_single.sh
N=134217728 B=16 IT=6 VARS="cs4 cs16 cur" bash tools/ab_batch16.sh
N=16777216 B=64 VARS="cs4 cs16 cur ss4 ss16" bash tools/ab_batch16.sh
VARS="ss16 ss4 cur" bash tools/ab_single.sh
