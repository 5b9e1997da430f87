#!/bin/bash
# Build libmathocr.so from the current sources with PATCH applied, into DIR, with the
# UNPATCHED tree's source hash baked in (engine.load_library accepts it beside the current
# sources): an A/B variant for the probes and bench (--lib DIR/libmathocr.so), never a
# product build.   Usage: tools/build_patch_variant.sh DIR PATCH [extra hipcc flags...]
set -e
OUT=$(realpath -m "$1"); PATCH=$(realpath "$2"); shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d /tmp/mocr_pv_XXXX)
mkdir -p "$SRC/pkg" "$SRC/include" "$OUT/obj"
cp -r "$ROOT/handwritten-math-ocr-api_amd/csrc" "$SRC/pkg/"
cp "$ROOT/include/mathocr.h" "$SRC/include/"
(cd "$SRC" && mkdir -p handwritten-math-ocr-api_amd && ln -s ../pkg/csrc handwritten-math-ocr-api_amd/csrc \
  && patch -s -p1 < "$PATCH")
cd "$SRC/pkg"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" \
    -c "$f" -o "$OUT/obj/$(basename "$f" .hip).o" &
done
wait
cd "$ROOT/handwritten-math-ocr-api_amd"
H=$(cat $(ls csrc/*.hip csrc/*.h | LC_ALL=C sort) ../include/mathocr.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* mocr_source_hash(void) { return "%s"; }\nextern "C" const char* mocr_build_tag(void) { return "ab:%s"; }\n' $H "build_patch_variant.sh $*" > "$OUT/obj/srchash.cpp"
g++ -O2 -fPIC -c "$OUT/obj/srchash.cpp" -o "$OUT/obj/srchash.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
rm -rf "$SRC"
echo "built $OUT/libmathocr.so with $(basename "$PATCH")"
