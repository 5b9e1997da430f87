#!/bin/bash
# decode attention: phase clocks (1 / 2 / 4 waves), parity, decode chain
set -o pipefail
O=gpurun_out/aw; mkdir -p $O
if [ -x tools/attn_ts ] && [ -f handwritten-math-ocr-api_amd/lib_var/ts/libmathocr.so ]; then
  for args in "cross 256 100" "self 256 16" "self 256 60" "self 256 120"; do
    for w in ${WAVES:-0}; do timeout -k 10 60 ./tools/attn_ts $args $w | head -2 | tail -2 || exit 1; done
  done
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "teacher_forced or b256_chain or config2 or eos or invariance or greedy or stop" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|PARITY" $O/tests.log | tail -5
timeout -k 10 180 python -u tools/decode_chain_probe.py --rows 256 --chains 1,2 --reps 2 2>&1 | grep rows_per_s || exit 1
