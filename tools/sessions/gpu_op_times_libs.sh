#!/bin/bash
# tools/op_times.py over several libmathocr.so builds, alternating twice:
#   tools/sessions/gpu_op_times_libs.sh TAG FILTER LIB...
mkdir -p gpurun_out
TAG=$1; F=$2; shift 2
O=gpurun_out/optimes_$TAG.log
: > $O
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib" >> $O
    timeout -k 10 180 python tools/op_times.py --lib $lib --variants production --filter $F >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu $O | grep -v "^op\|^total"
