#!/bin/bash
# (1) GPU parity suite on production (fused stage-3 attention at every batch).  (2) fold
# GEMMs loading A as 8 rows x 128 B per wave instruction (a8) and 32-row logits tiles above
# 256 rows (lbm32), development builds (tools/build_dev.sh), vs production: decode chains and
# bench, interleaved.  (3) the parity suite on each (its library copied over lib/ on this
# scratch box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04y; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in production a8 lbm32 production a8 lbm32; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512,640 --chains 1,2 --reps 2 $(lib $L) > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-150
done
for L in production a8 lbm32 production a8 lbm32; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_libmathocr.so
for L in a8 lbm32; do
  cp handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so $P
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
    > $O/tests_$L.log 2>&1 || { echo "TESTS $L FAILED"; tail -40 $O/tests_$L.log; cp /tmp/prod_libmathocr.so $P; exit 1; }
  tail -2 $O/tests_$L.log
done
cp /tmp/prod_libmathocr.so $P
echo done
