#!/bin/bash
# Round 5: mlp384 on 8 waves (two per SIMD, 16 rows each; lib_var/m8) vs production (4 waves,
# one per SIMD). Bitwise memory check, per-op times, parity tests on the variant, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07i; mkdir -p $O
V=handwritten-math-ocr-api_amd/lib_var/m8/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_var.npy --lib $V >> $O/mem.log 2>&1 || { echo "MEM VAR FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_var.npy'); print('m8 memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
rm -f $O/*.npy
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production m8 production m8; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s3.mlp $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "mlp" $O/ops_$L.log
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_lib.so; cp $V $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched" > $O/tests_m8.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests_m8.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests m8: $(tail -1 $O/tests_m8.log)"; cp /tmp/prod_lib.so $P
for L in production m8 production m8; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
