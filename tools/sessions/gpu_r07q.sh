#!/bin/bash
# Round 5: stem16w with X leaving through a 6 KB LDS slice per wave as whole 16-B lanes
# (lib_var/stemlo) vs production (three 8-B stores per lane, 24 B apart). Bitwise memory,
# stem time, parity tests on the variant, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07q; mkdir -p $O
V=handwritten-math-ocr-api_amd/lib_var/stemlo/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_var.npy --lib $V >> $O/mem.log 2>&1 || { echo "MEM VAR FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_var.npy'); print('stemlo memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
rm -f $O/*.npy
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production stemlo production stemlo; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter stem $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "stem" $O/ops_$L.log
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_lib.so; cp $V $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched" > $O/tests_stemlo.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests_stemlo.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests stemlo: $(tail -1 $O/tests_stemlo.log)"; cp /tmp/prod_lib.so $P
for L in production stemlo production stemlo; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
