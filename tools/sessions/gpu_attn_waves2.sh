#!/bin/bash
# decode chains with 2-wave (production) vs 4-wave attention, alternating, then the bench pair
set -o pipefail
for rep in 1 2; do
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/w4/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 180 python -u tools/decode_chain_probe.py --lib $lib --rows 256 --chains 1,2 --reps 2 2>&1 | grep rows_per_s || exit 1
done
done
