#!/bin/bash
# The self-attention cache in int16 with per-(row, head, key) scales (production) vs fp24
# (HEAD, base): the GPU parity suite (incl. the fp24 variant and a NaN in the self-attention
# keys), decode chains and the bench, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05b; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -h "PARITY_RECORD\|teacher-forced logits" $O/tests.log | cut -c1-250 | head -40
for L in production base production base; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512,640 --chains 1,2 --reps 2 $(lib $L) > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-150
done
for L in production base production base; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
echo done
