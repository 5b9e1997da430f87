#!/bin/bash
# stage 3's norm1 + qkv in one kernel (lngemm384): stage parity, encoder op times vs the
# unfused pair, the B = 256 chain fixture
set -o pipefail
O=gpurun_out/lng; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "encoder_stages or b256_chain or bf16_encoder_modes" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|PARITY" $O/tests.log | tail -6
timeout -k 10 300 python tools/op_times.py --batch 256 --variants production,unfused_ln_gemm --filter s3.,merge 2>&1 | grep -v amdgpu.ids || exit 1
