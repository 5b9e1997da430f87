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
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmathocr.so" "$OUT"/obj/*.o -ldl
echo "built $OUT/libmathocr.so"
