#!/bin/bash
# Encoder A/B on one box: memory and 8-step logits at 256 images bitwise against lib_var/head
# (the previous commit; VAR=NAME: lib_var/NAME), then the driver-form bench, lib/ against it, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-abbit}; mkdir -p $O
L=handwritten-math-ocr-api_amd/lib_var
timeout -k 10 180 python tools/mem_dump.py /tmp/cur.npy --batch 256 --decode 8 > $O/dump.log 2>&1 || { echo "DUMP FAILED"; tail $O/dump.log; exit 1; }
timeout -k 10 180 python tools/mem_dump.py /tmp/head.npy --batch 256 --decode 8 --lib $L/${VAR:-head}/libmathocr.so >> $O/dump.log 2>&1 || { echo "DUMP HEAD FAILED"; tail $O/dump.log; exit 1; }
python -c "
import numpy as np
a=np.load('/tmp/cur.npy'); b=np.load('/tmp/head.npy')
print('memory bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max|d|', float(np.abs(a-b).max()))
a=np.load('/tmp/cur_logits.npy'); b=np.load('/tmp/head_logits.npy')
print('logits bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)))
" | tee $O/bitwise.txt
TAG=${TAG:-abbit} bash tools/sessions/gpu_ab.sh ${VAR:-head} "$@"
