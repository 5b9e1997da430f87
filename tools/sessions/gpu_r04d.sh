#!/bin/bash
# A/B of the decode step vs rows per chain: current tree against lib_var/base (HEAD), then
# the GPU suite on the current tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04d; mkdir -p $O
for L in new base; do
  A=""; [ $L = base ] && A="--lib handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so"
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,320,384,512 --chains 1 --reps 2 $A > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512 --chains 2 --reps 2 $A > $O/rows2_$L.log 2>&1 \
    || { echo "ROWS2 $L FAILED"; tail $O/rows2_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log $O/rows2_$L.log | cut -c1-140
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
