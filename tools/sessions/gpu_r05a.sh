#!/bin/bash
# Stage 4's fused no-proj attention (MOCR_VARIANT_S4_FUSED_ATTN) on fragment-major W_qkv
# (s4fm, a development build) vs the unfused stage-4 sequence: per-op times at 512 and 64
# images per encode; the parity suite on the s4fm library (copied over lib/ on this box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05a; mkdir -p $O
L="--lib handwritten-math-ocr-api_amd/lib_var/s4fm/libmathocr.so"
for B in 512 64; do
  timeout -k 10 300 python -u tools/op_times.py --batch $B --encodes 3 --variants production,s4_fused_attn --filter s4. $L > $O/ops$B.log 2>&1 \
    || { echo "OPS $B FAILED"; tail $O/ops$B.log; exit 1; }
  echo "== B $B"; cat $O/ops$B.log | grep -v amdgpu.ids
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_libmathocr.so && cp handwritten-math-ocr-api_amd/lib_var/s4fm/libmathocr.so $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests_s4fm.log 2>&1 || { echo "TESTS S4FM FAILED"; tail -40 $O/tests_s4fm.log; cp /tmp/prod_libmathocr.so $P; exit 1; }
cp /tmp/prod_libmathocr.so $P
tail -2 $O/tests_s4fm.log
echo done
