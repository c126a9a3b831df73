# Build a diagnostic / A-B variant of libfedcodec.so: tools/mkvar.sh <name> [-DFLAG=...]...
# -> tools/variants/lib_<name>.so (git-ignored; travels to the GPU box with the tree).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/tools/variants"
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -shared --offload-arch=gfx950 \
  -Wno-unused-function "$@" -o "$ROOT/tools/variants/lib_$NAME.so" "$ROOT/openmsftl_amd/csrc/fedcodec.hip"
echo "built tools/variants/lib_$NAME.so ($*)"
