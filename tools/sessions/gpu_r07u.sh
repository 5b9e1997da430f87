#!/bin/bash
# Round 5: int16 cross-attention on 16-B loads (dec_xattn16_kernel: 4 lanes per key row; xa1 =
# 2 waves / 5 passes, xa2 = 3 waves / 3 passes over the 144 memory keys) vs production
# (dec_foldattn_kernel, 8 lanes of 8-B loads). Not bitwise (another summation order): the
# decode parity tests on each variant, decode chains at 512 / 640 rows, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07u; mkdir -p $O
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
cp $P /tmp/prod_lib.so
for V in xa1 xa2; do
  cp handwritten-math-ocr-api_amd/lib_var/$V/libmathocr.so $P
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_conditioning.py -x -q --timeout 300 --timeout-method thread \
    > $O/tests_$V.log 2>&1 || { echo "TESTS $V FAILED"; tail -30 $O/tests_$V.log; cp /tmp/prod_lib.so $P; exit 1; }
  echo "tests $V: $(tail -1 $O/tests_$V.log)"
done
cp /tmp/prod_lib.so $P
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production xa1 xa2 production xa1 xa2; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 1 --reps 2 $(lib $L) > $O/dec_$L.log 2>&1 || { echo "DEC $L FAILED"; tail $O/dec_$L.log; exit 1; }
  echo "== $L"; grep -E "rows_per_s|us" $O/dec_$L.log | cut -c1-150 | tail -2
done
for L in production xa1 xa2 production xa1 xa2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
