#!/bin/bash
# Round 6: the fold GEMMs' XCD-local tile map (decwide.hip MOCR_FOLD_XCD_COLS = 1 / 2 / 4
# column groups) against the column-fastest map: bitwise logits of a 640-row chain, then
# one and two 640-row chains' us per step, interleaved base / variant runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s6b; mkdir -p $O
L=handwritten-math-ocr-api_amd/lib_var
timeout -k 10 120 python tools/mem_dump.py /tmp/base.npy --batch 640 --decode 16 > $O/dump.log 2>&1 || { echo "DUMP FAILED"; tail $O/dump.log; exit 1; }
for v in xc1 xc2 xc4; do
  timeout -k 10 120 python tools/mem_dump.py /tmp/$v.npy --batch 640 --decode 16 --lib $L/$v/libmathocr.so >> $O/dump.log 2>&1 || { echo "DUMP $v FAILED"; tail $O/dump.log; exit 1; }
  python -c "
import numpy as np
a=np.load('/tmp/base_logits.npy'); b=np.load('/tmp/${v}_logits.npy')
print('$v logits bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'ids', np.array_equal(np.load('/tmp/base_ids.npy'), np.load('/tmp/${v}_ids.npy')))
" | tee -a $O/bitwise.txt
done
for lib in base xc2 xc4 xc1 base xc2; do
  arg=""; [ $lib != base ] && arg="--lib $L/$lib/libmathocr.so"
  echo "== $lib" >> $O/chain.log
  timeout -k 10 200 python tools/decode_chain_probe.py --rows 640 --chains 1,2 --reps 3 $arg >> $O/chain.log 2>&1 || { echo "CHAIN $lib FAILED"; tail $O/chain.log; exit 1; }
done
grep -E '^==|rows' $O/chain.log
echo done
