# Build librwkvtts.so of git revision REV into build/rev/NAME/ (same-box A/B timing against the
# working tree through RWKVTTS_LIB). Usage: bash tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build/rev_src/$NAME
rm -rf "$D"; mkdir -p "$D" "$R/build/rev/$NAME"
git -C "$R" archive "$REV" rwkv-tts-rs_amd/csrc include | tar -x -C "$D"
make -C "$D/rwkv-tts-rs_amd/csrc" -j8 OUT="$R/build/rev/$NAME/librwkvtts.so" OBJDIR="$D/obj" > "$D/build.log" 2>&1
echo "built $R/build/rev/$NAME/librwkvtts.so"
