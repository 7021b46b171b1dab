# Build librwkvtts.so of git revision REV with a source edit applied into ab_libs/NAME/.
# Usage: bash tools/build_rev_variant.sh REV NAME [PYTHON_EDIT_SCRIPT]
set -e
REV=$1; NAME=$2; EDIT=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build/var_src/$NAME
rm -rf "$D"; mkdir -p "$D" "$R/ab_libs/$NAME"
git -C "$R" archive "$REV" rwkv-tts-rs_amd/csrc include | tar -x -C "$D"
[ -n "$EDIT" ] && (cd "$D/rwkv-tts-rs_amd/csrc" && python3 "$R/$EDIT")
make -C "$D/rwkv-tts-rs_amd/csrc" -j8 OUT="$R/ab_libs/$NAME/librwkvtts.so" OBJDIR="$D/obj" > "$D/build.log" 2>&1
echo "built ab_libs/$NAME/librwkvtts.so"
