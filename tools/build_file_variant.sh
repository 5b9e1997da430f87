#!/bin/bash
# A/B build of libmathocr.so in which ONE source file gets extra compile flags (the other
# objects are the in-tree production build's).  Usage: tools/build_file_variant.sh DIR FILE FLAGS...
# e.g. tools/build_file_variant.sh lib_var/noslp_mlp mlp.hip -fno-slp-vectorize
set -e
OUT=$1; F=$2; shift 2
cd "$(dirname "$0")/../handwritten-math-ocr-api_amd"
make -j8 >/dev/null
mkdir -p "$OUT/obj"
cp build/*.o "$OUT/obj/"
H=$(cat $(ls csrc/*.hip csrc/*.h | LC_ALL=C sort) ../include/mathocr.h | sha256sum | cut -c1-16)
printf 'extern "C" const char* mocr_source_hash(void) { return "%s"; }\nextern "C" const char* mocr_build_tag(void) { return "ab:%s"; }\n' $H "build_file_variant.sh $F $*" > "$OUT/obj/srchash.cpp"
g++ -O2 -fPIC -c "$OUT/obj/srchash.cpp" -o "$OUT/obj/srchash.o"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" \
  -c "csrc/$F" -o "$OUT/obj/$(basename "$F" .hip).o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
echo "built $OUT/libmathocr.so ($F: $*)"
