# Same-box A/B of two source trees (e.g. an ABI change): each probe runs from tree A and tree B,
# alternating A B B A, every line tagged with its tree.
#   gpurun -- 'bash tools/ab_tree.sh <out.jsonl> <treeA> <treeB> "<probe args>" ...'
set -e
OUT=$1; A=$2; B=$3; shift 3
mkdir -p "$(dirname "$OUT")"
run() {
  local tree=$1 probe=$2
  (cd "$tree" && timeout -k 10 300 python -u tools/kbench.py $probe --tag "$tree") | tail -1 | tee -a "$OUT"
}
for p in "$@"; do run "$A" "$p"; run "$B" "$p"; done
for p in "$@"; do run "$B" "$p"; run "$A" "$p"; done
