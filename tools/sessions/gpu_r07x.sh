#!/bin/bash
# Round 5: the stage-4 window attention's O planes as 16-B stores (lane pairs trade halves;
# lib_var/watt16) vs production (two 8-B stores per plane). Bitwise memory, s4.wattn time,
# parity tests on the variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07x; mkdir -p $O
V=handwritten-math-ocr-api_amd/lib_var/watt16/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_var.npy --lib $V >> $O/mem.log 2>&1 || { echo "MEM VAR FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_var.npy'); print('watt16 memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
rm -f $O/*.npy
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production watt16 production watt16; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s4.wattn $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "wattn" $O/ops_$L.log
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_lib.so; cp $V $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched or window_rows or pixel_rows" > $O/tests_watt16.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests_watt16.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests watt16: $(tail -1 $O/tests_watt16.log)"; cp /tmp/prod_lib.so $P
echo done
