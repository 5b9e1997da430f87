#!/bin/bash
# Build libmathocr.so from a development copy of the sources (SRCDIR holding pkg/csrc/ and
# include/, the repository's relative layout) into DIR, with the CURRENT tree's source hash baked in, so that
# engine.load_library(DIR/libmathocr.so) accepts it beside the current sources: an A/B
# probe build, never a product build.   Usage: tools/build_dev.sh SRCDIR DIR [FLAGS...]
set -e
SRC=$(realpath "$1"); OUT=$(realpath -m "$2"); shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT/obj"
cd "$SRC/pkg"
pids=()
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" \
    -c "$f" -o "$OUT/obj/$(basename "$f" .hip).o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done  # set -e: a failed compile ends the build
cd "$ROOT/handwritten-math-ocr-api_amd"
H=$(cat $(ls csrc/*.hip csrc/*.h | LC_ALL=C sort) ../include/mathocr.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* mocr_source_hash(void) { return "%s"; }\nextern "C" const char* mocr_build_tag(void) { return "ab:%s"; }\n' $H "build_dev.sh $*" > "$OUT/obj/srchash.cpp"
g++ -O2 -fPIC -c "$OUT/obj/srchash.cpp" -o "$OUT/obj/srchash.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
echo "built $OUT/libmathocr.so from $SRC"
