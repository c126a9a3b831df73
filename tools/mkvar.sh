# Build a diagnostic / A-B variant of libfedcodec.so: tools/mkvar.sh <name> [FC_NAME=VALUE]...
# [-DFLAG]...  FC_NAME=VALUE rewrites the tuned constant `constexpr int FC_NAME = ...;` in a
# copy of the sources (the product source carries no -D switches); -D flags (FC_TRACE,
# FC_DEBUG_BUILD) go to hipcc.  -> tools/variants/lib_<name>.so (git-ignored; travels to the
# GPU box with the tree).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
exec bash "$ROOT/tools/patchvar.sh" "$NAME" "$ROOT/tools/edits/none.py" "$@"
