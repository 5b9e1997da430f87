#!/bin/bash
# Decode-step A/B on one box: bitwise logits of a 640-row, 16-step chain against lib/, then
# one and two 640-row chains (us per step / rows per s), interleaved with lib/.
#   TAG=... bash tools/sessions/gpu_dec_ab.sh NAME [NAME...]   (handwritten-math-ocr-api_amd/lib_var/NAME)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-decab}; mkdir -p $O
L=handwritten-math-ocr-api_amd/lib_var
timeout -k 10 150 python tools/mem_dump.py /tmp/base.npy --batch 640 --decode 16 > $O/dump.log 2>&1 || { echo "DUMP FAILED"; tail $O/dump.log; exit 1; }
for v in "$@"; do
  timeout -k 10 150 python tools/mem_dump.py /tmp/$v.npy --batch 640 --decode 16 --lib $L/$v/libmathocr.so >> $O/dump.log 2>&1 || { echo "DUMP $v FAILED"; tail $O/dump.log; exit 1; }
  python -c "
import numpy as np
a=np.load('/tmp/base_logits.npy'); b=np.load('/tmp/${v}_logits.npy')
print('$v logits bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max|d|', float(np.abs(a-b).max()), 'ids', np.array_equal(np.load('/tmp/base_ids.npy'), np.load('/tmp/${v}_ids.npy')))
" | tee -a $O/bitwise.txt
done
for rep in 1 2; do
  for v in base "$@"; do
    arg=""; [ $v != base ] && arg="--lib $L/$v/libmathocr.so"
    echo "== $v $rep" >> $O/chain.log
    timeout -k 10 200 python tools/decode_chain_probe.py --rows 640 --chains 1,2 --reps 3 $arg >> $O/chain.log 2>&1 || { echo "CHAIN $v FAILED"; tail $O/chain.log; exit 1; }
  done
done
grep -E '^==|rows' $O/chain.log | python3 -c "
import sys, json
cur=None
for l in sys.stdin:
    if l.startswith('=='): cur=l.strip()[3:]; continue
    d=json.loads(l); print(cur, d['chains'], round(d['us_per_step_per_chain'],1), round(d['rows_per_s']))"
echo done
