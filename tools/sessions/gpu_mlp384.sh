#!/bin/bash
# Stage-3 fused MLP: encoder parity (every bf16 variant) then per-op times fused vs
# unfused at B = 64 and 256.  Usage: tools/sessions/gpu_mlp384.sh TAG
set -o pipefail
mkdir -p gpurun_out
T=${1:-mlp384}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "encoder_stages or bf16_encoder_modes or memory_matches or greedy_ids" > gpurun_out/${T}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for B in 64 256; do
  timeout -k 10 240 python tools/op_times.py --batch $B --variants production,unfused_mlp --filter s3. \
    > gpurun_out/${T}_optimes_b$B.log 2>&1 || { echo "OPTIMES FAILED"; tail -20 gpurun_out/${T}_optimes_b$B.log; exit 1; }
  grep -v amdgpu gpurun_out/${T}_optimes_b$B.log
done
