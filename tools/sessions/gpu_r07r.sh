#!/bin/bash
# Round 5: ln_group_kernel with its bf16 hi / lo planes staged in LDS and stored as whole
# 16-B lanes (lib_var/lnlo) vs production (8-B stores per lane, 2F B apart). Bitwise memory,
# merge / stage-4 norm times, parity tests on the variant (all encoder variants), bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07r; mkdir -p $O
V=handwritten-math-ocr-api_amd/lib_var/lnlo/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_var.npy --lib $V >> $O/mem.log 2>&1 || { echo "MEM VAR FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_var.npy'); print('lnlo memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
rm -f $O/*.npy
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production lnlo production lnlo; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter merge,s4.ln $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "ln" $O/ops_$L.log
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_lib.so; cp $V $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched or window_rows or pixel_rows" > $O/tests_lnlo.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests_lnlo.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests lnlo: $(tail -1 $O/tests_lnlo.log)"; cp /tmp/prod_lib.so $P
for L in production lnlo production lnlo; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
