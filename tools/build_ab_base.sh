#!/bin/bash
# Build libmathocr.so from the sources of git revision REV (default HEAD) into DIR, with the
# CURRENT tree's source hash baked in, so that engine.load_library(DIR/libmathocr.so)
# accepts it beside the current sources: an A/B baseline for the probes (tools/*probe*.py
# --lib), never a product build.   Usage: tools/build_ab_base.sh DIR [REV]
set -e
OUT=$(realpath -m "$1"); REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d /tmp/mocr_ab_XXXX)
mkdir -p "$SRC/pkg/csrc" "$SRC/include" "$OUT/obj"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" handwritten-math-ocr-api_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$SRC/pkg/csrc/$(basename $f)"
done
git -C "$ROOT" show "$REV:include/mathocr.h" > "$SRC/include/mathocr.h"
cd "$SRC/pkg"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include \
    -c "$f" -o "$OUT/obj/$(basename "$f" .hip).o" &
done
wait
cd "$ROOT/handwritten-math-ocr-api_amd"
H=$(cat $(ls csrc/*.hip csrc/*.h | LC_ALL=C sort) ../include/mathocr.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* mocr_source_hash(void) { return "%s"; }\nextern "C" const char* mocr_build_tag(void) { return "ab:%s"; }\n' $H "build_ab_base.sh $*" > "$OUT/obj/srchash.cpp"
g++ -O2 -fPIC -c "$OUT/obj/srchash.cpp" -o "$OUT/obj/srchash.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
rm -rf "$SRC"
echo "built $OUT/libmathocr.so from $REV"
