#!/bin/bash
# int16 cross-attention K/V: parity tests, then decode-step A/B against fp24 cross K/V
set -o pipefail
mkdir -p gpurun_out/kvx16
O=gpurun_out/kvx16
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "teacher_forced or b256_chain or config2" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|PARITY" $O/tests.log | tail -12
for rep in 1 2; do
for v in "" cross_kv_f24; do
  echo "== variant '$v'"
  timeout -k 10 180 python -u tools/decode_chain_probe.py --rows 256 --chains 1,2 --reps 2 --variant "$v" 2>&1 | grep -v "^$" | tail -4 || exit 1
done
done
