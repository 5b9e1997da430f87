#!/bin/bash
# Stage 3 on the fused norm1 + qkv + W-MSA + proj + residual kernel with its k-loops
# unrolled by 2 at C = 384 (fp384u2, no spills; a development build) vs production: per-op
# times of a 512-image encode, bench, interleaved; the parity suite on fp384u2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05f; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production fp384u2 production fp384u2; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s3. $(lib $L) > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "s3|total" $O/ops_$L.log
done
for L in production fp384u2 production fp384u2; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_libmathocr.so && cp handwritten-math-ocr-api_amd/lib_var/fp384u2/libmathocr.so $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests_fp384u2.log 2>&1 || { echo "TESTS MLPPF FAILED"; tail -40 $O/tests_fp384u2.log; cp /tmp/prod_libmathocr.so $P; exit 1; }
cp /tmp/prod_libmathocr.so $P
tail -1 $O/tests_fp384u2.log
echo done
