#!/bin/bash
# The stem kernel requesting the next token's pixels before this token's math (stempf, a
# development build) vs production: per-op times at 512 and 64 images, bench, interleaved;
# the parity suite on stempf (copied over lib/ on this box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05h; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production stempf production stempf; do
  for B in 512 64; do
    timeout -k 10 300 python -u tools/op_times.py --batch $B --encodes 3 --variants production --filter stem $(lib $L) > $O/ops${B}_$L.log 2>&1 \
      || { echo "OPS $L FAILED"; tail $O/ops${B}_$L.log; exit 1; }
    echo "== $L B $B"; grep -E "stem" $O/ops${B}_$L.log
  done
done
for L in production stempf production stempf; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_libmathocr.so && cp handwritten-math-ocr-api_amd/lib_var/stempf/libmathocr.so $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests_stempf.log 2>&1 || { echo "TESTS STEMPF FAILED"; tail -40 $O/tests_stempf.log; cp /tmp/prod_libmathocr.so $P; exit 1; }
cp /tmp/prod_libmathocr.so $P
tail -1 $O/tests_stempf.log
echo done
