# Build an A/B variant of libfedcodec.so from a patched copy of the sources (experiments that
# are not a tuned constant): tools/patchvar.sh <name> <python-file-with-edits> [FC_NAME=V]... [-DFLAG]...
# The edits file defines edits = [(path relative to openmsftl_amd/csrc, old, new), ...].
# -> tools/variants/lib_<name>.so (git-ignored; travels to the GPU box with the tree).
# FC_NAME=VALUE arguments rewrite `constexpr int FC_NAME = ...;`; other arguments go to hipcc.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EDITS=$2; shift 2
CONSTS=(); FLAGS=()
for a in "$@"; do
  case "$a" in FC_*=*) CONSTS+=("$a") ;; *) FLAGS+=("$a") ;; esac
done
TMP=$(mktemp -d)
mkdir -p "$TMP/openmsftl_amd" "$TMP/include" "$ROOT/tools/variants"
cp -r "$ROOT/openmsftl_amd/csrc" "$TMP/openmsftl_amd/"
cp "$ROOT/include/fedcodec.h" "$TMP/include/"
python3 - "$TMP/openmsftl_amd/csrc" "$EDITS" "${CONSTS[@]}" <<'PY'
import glob, re, runpy, sys
d, f = sys.argv[1], sys.argv[2]
for path, old, new in runpy.run_path(f)["edits"]:
    p = f"{d}/{path}"
    s = open(p).read()
    assert old in s, (path, old[:60])
    open(p, "w").write(s.replace(old, new))
for kv in sys.argv[3:]:
    name, val = kv.split("=", 1)
    hits = 0
    for p in glob.glob(f"{d}/*.h") + glob.glob(f"{d}/*.hip"):
        s = open(p).read()
        s2, c = re.subn(rf"constexpr int {name} = [^;]+;", f"constexpr int {name} = {val};", s)
        hits += c
        if c:
            open(p, "w").write(s2)
    assert hits == 1, (name, hits)
PY
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -shared --offload-arch=gfx950 \
  -Wno-unused-function "${FLAGS[@]}" -o "$ROOT/tools/variants/lib_$NAME.so" "$TMP/openmsftl_amd/csrc/fedcodec.hip"
rm -rf "$TMP"
echo "built tools/variants/lib_$NAME.so ($EDITS $*)"
