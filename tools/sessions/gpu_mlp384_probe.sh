#!/bin/bash
# Stage-3 fused MLP: encoder parity, then s3.mlp at B = 256 for the production build and
# the timing probes in lib_var/ (tools/build_variant.sh DIR -DMOCR_MLP384_PROBE=N).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "encoder_stages or bf16_encoder_modes or memory_matches or greedy_ids" > gpurun_out/mlp384_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 gpurun_out/mlp384_tests.log; exit 1; }
tail -1 gpurun_out/mlp384_tests.log
for lib in handwritten-math-ocr-api_amd/lib/libmathocr.so handwritten-math-ocr-api_amd/lib_var/*/libmathocr.so; do
  echo "== $lib"
  timeout -k 10 120 python tools/op_times.py --lib $lib --batch ${B:-256} --variants production --filter s3.mlp 2>&1 | grep "s3.mlp" || exit 1
done
