#!/bin/bash
# -fno-slp-vectorize (no v_pk_*_f32 beside the MFMAs) vs production: encoder op times and
# the decode chain, alternating
set -o pipefail
for rep in 1 2; do
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/noslp/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 120 python tools/op_times.py --lib $lib --batch 256 --variants production 2>&1 | grep -v amdgpu.ids | grep -v "^op" || exit 1
done
done
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/noslp/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 180 python -u tools/decode_chain_probe.py --lib $lib --rows 256 --chains 1,2 --reps 2 2>&1 | grep rows_per_s || exit 1
done
