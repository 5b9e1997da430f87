#!/bin/bash
# Build libmathocr.so with extra compile flags into another directory, for A/B probes
# (tools/pipeline_probe.py --lib DIR/libmathocr.so).  Usage: tools/build_variant.sh DIR FLAGS...
set -e
OUT=$1; shift
cd "$(dirname "$0")/../handwritten-math-ocr-api_amd"
mkdir -p "$OUT/obj"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" \
    -c "$f" -o "$OUT/obj/$(basename "$f" .hip).o" &
done
wait
# the source hash the Makefile bakes in (engine.load_library checks it)
H=$(cat $(ls csrc/*.hip csrc/*.h | LC_ALL=C sort) ../include/mathocr.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* mocr_source_hash(void) { return "%s"; }\nextern "C" const char* mocr_build_tag(void) { return "ab:%s"; }\n' $H "build_variant.sh $*" > "$OUT/obj/srchash.cpp"
g++ -O2 -fPIC -c "$OUT/obj/srchash.cpp" -o "$OUT/obj/srchash.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
echo "built $OUT/libmathocr.so"
