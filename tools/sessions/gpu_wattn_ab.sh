#!/bin/bash
# window attention V loads: LDS transpose (production) vs scalar gathers, alternating
set -o pipefail
for rep in 1 2 3; do
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/vg/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 120 python tools/op_times.py --lib $lib --batch 256 --variants production --filter s3.wattn,s4.wattn 2>&1 | grep wattn || exit 1
done
done
