set -e
N=16777216 B=64 VARS="ntld" bash tools/ab_batch16.sh
N=134217728 B=16 IT=6 VARS="ntld" bash tools/ab_batch16.sh
VARS="ntld" bash tools/ab_single.sh
N=134217728 B=16 IT=6 VARS="ntld" bash tools/ab_batch16.sh
