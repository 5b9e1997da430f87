#!/bin/bash
# Window attention (stages 3-4) with unconditional operand loads vs HEAD: per-op times at a
# 512-image encode, the encoder parity tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04n; mkdir -p $O
for L in new base new base; do
  A=""; [ $L = base ] && A="--lib handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so"
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s3.,s4. $A > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "wattn|total" $O/ops_$L.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
