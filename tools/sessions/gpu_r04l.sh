#!/bin/bash
# Decode attention on 4 waves per (row, head) for 41-160 keys (-DMOCR_ATTN_WAVES=4) vs the
# default 2, at the bench's chain lengths.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04l; mkdir -p $O
for L in production aw4 production aw4; do
  A=""; [ $L = aw4 ] && A="--lib handwritten-math-ocr-api_amd/lib_var/aw4/libmathocr.so"
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 1,2 --reps 2 $A > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-140
done
echo done
