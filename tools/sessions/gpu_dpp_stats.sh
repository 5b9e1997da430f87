#!/bin/bash
# LN-statistics merge trees on DPP: decode parity, fold GEMM phase clocks, decode chain
set -o pipefail
O=gpurun_out/dpp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "teacher_forced or b256_chain or config2 or unfolded or beam or narrow" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 60 ./tools/fold_ts 256 256 256 && timeout -k 10 60 ./tools/fold_ts 256 512 768 || exit 1
timeout -k 10 180 python -u tools/decode_chain_probe.py --rows 256 --chains 1,2 --reps 2 2>&1 | grep rows_per_s || exit 1
