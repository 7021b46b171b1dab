# Build the working tree's librwkvtts.so with a source edit applied into ab_libs/NAME/ (same-box
# A/B of an experiment without touching the tree). Usage:
#   bash tools/build_variant.sh NAME PYTHON_EDIT_SCRIPT [EXTRA_FLAGS]
# The edit script runs with cwd = the copied rwkv-tts-rs_amd/csrc.
set -e
NAME=$1; EDIT=$2; EXTRA=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build/var_src/$NAME
rm -rf "$D"; mkdir -p "$D/rwkv-tts-rs_amd" "$R/ab_libs/$NAME"
cp -r "$R/rwkv-tts-rs_amd/csrc" "$D/rwkv-tts-rs_amd/"; cp -r "$R/include" "$D/"
rm -f "$D"/rwkv-tts-rs_amd/csrc/*.o
(cd "$D/rwkv-tts-rs_amd/csrc" && python3 "$R/$EDIT")
make -C "$D/rwkv-tts-rs_amd/csrc" -j8 OUT="$R/ab_libs/$NAME/librwkvtts.so" OBJDIR="$D/obj" EXTRA="$EXTRA" > "$D/build.log" 2>&1
echo "built ab_libs/$NAME/librwkvtts.so"
