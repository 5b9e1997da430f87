#!/bin/bash
# Fold GEMMs on 4 waves (-DMOCR_FOLD_WAVES=4) and the logits on 8 (-DMOCR_LOGITS_WAVES=8)
# against the defaults (8, 4) at the bench's chain lengths, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04m; mkdir -p $O
for L in production fw4 lw8 production fw4 lw8; do
  A=""; [ $L != production ] && A="--lib handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so"
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 1,2 --reps 2 $A > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-140
done
echo done
