# Builds the library of a committed revision (default HEAD) out of tree for A/B timing:
# build/rev_src/<rev> (git archive) -> build/ab/lib_<rev>.so. Usage: bash tools/build_rev.sh [rev]
set -e
REV=${1:-HEAD}
NAME=$(git rev-parse --short "$REV")
DST=build/rev_src/$NAME
rm -rf "$DST" && mkdir -p "$DST" build/ab
git archive "$REV" rwkv-tts-rs_amd/csrc include | tar -x -C "$DST"
make -C "$DST/rwkv-tts-rs_amd/csrc" -j8 > /dev/null
cp "$DST/rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" "build/ab/lib_$NAME.so"
echo "build/ab/lib_$NAME.so"
