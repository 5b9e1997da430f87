#!/bin/bash
# int16 cross K/V quantised in the crosskv GEMM epilogue: parity subset, encoder op times, bench
set -o pipefail
O=gpurun_out/kvx16b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  -k "teacher_forced or b256_chain or config2 or eos" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|PARITY" $O/tests.log | tail -12
timeout -k 10 200 python tools/op_times.py --batch 256 --variants production --filter crosskv,memkv 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
