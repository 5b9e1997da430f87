#!/bin/bash
# Round 5: the rest of the suite (sharded bench test), the default bench on the new tree,
# and the 32 x 16 vectorised fold epilogue (lib_var/v4b) vs production: decode chains and
# the bench, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06c; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v -rP --timeout 280 --timeout-method thread \
  > $O/tests_sharded.log 2>&1 || { echo "SHARDED FAILED"; tail -40 $O/tests_sharded.log; exit 1; }
tail -1 $O/tests_sharded.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "BENCH FAILED"; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_ratio'))"
for L in production v4b production v4b; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512,640 --chains 1,2 --reps 2 $(lib $L) > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log | cut -c1-150
done
for L in production v4b production v4b; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L"; python -c "import json; d=json.load(open('$O/bench20_$L.json')); print(d['value'])"
done
echo done
