#!/bin/bash
# Fold GEMM epilogue on 4 columns per thread extended to the 32 x 16 tiles (the y / z GEMMs
# of 256-row chains; v4b, a development build) vs production: parity suite on v4b (copied
# over lib/ on this box), decode chains and bench, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05j; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_libmathocr.so && cp handwritten-math-ocr-api_amd/lib_var/v4b/libmathocr.so $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests_v4b.log 2>&1 || { echo "TESTS V4EP FAILED"; tail -40 $O/tests_v4b.log; cp /tmp/prod_libmathocr.so $P; exit 1; }
cp /tmp/prod_libmathocr.so $P
tail -1 $O/tests_v4b.log
grep -h "PARITY_RECORD" $O/tests_v4b.log | cut -c1-200 | head -12
for L in production v4b production v4b; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512,640 --chains 1,2 --reps 2 $(lib $L) > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-150
done
for L in production v4b production v4b; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
echo done
