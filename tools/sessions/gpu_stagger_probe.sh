#!/bin/bash
# GEMM epilogue-stagger probe: s3 / s4 / merge GEMMs at B = 256, production vs lib_var builds
set -o pipefail
for rep in 1 2; do
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/*/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 120 python tools/op_times.py --lib $lib --batch 256 --variants production --filter s3.qkv,s3.proj,s4.,merge 2>&1 | grep -v amdgpu | grep -v "^op" || exit 1
done
done
