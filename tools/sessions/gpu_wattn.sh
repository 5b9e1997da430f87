#!/bin/bash
# stage 3/4 window attention: parity (stage maps, the B = 256 chain fixture), op times
set -o pipefail
O=gpurun_out/wattn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "encoder_stages or b256_chain or pixel_rows or bf16_encoder_modes" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|PARITY" $O/tests.log | tail -4
timeout -k 10 300 python tools/op_times.py --batch 256 --variants production --filter s3.wattn,s4.wattn 2>&1 | grep -v amdgpu.ids || exit 1
