#!/bin/bash
# (1) stage-1/2 MLP from packed chunk images and the stage-3 no-proj attention (B < 128) on
# fragment-major W_qkv (production) vs HEAD (base): per-op times of 512- and 64-image
# encodes, interleaved.  (2) the GPU parity suite.  (3) bench A/B incl. config2_literal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04v; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in base production base production; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.,s2. $(lib $L) > $O/ops512_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops512_$L.log; exit 1; }
  timeout -k 10 300 python -u tools/op_times.py --batch 64 --encodes 5 --variants production $(lib $L) > $O/ops64_$L.log 2>&1 \
    || { echo "OPS64 $L FAILED"; tail $O/ops64_$L.log; exit 1; }
  echo "== $L"; grep -E "mlp|attn|total" $O/ops512_$L.log; grep -E "s3.attn|total" $O/ops64_$L.log
done
for L in base production base production; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json,sys; d=json.load(open('$O/bench_$L.json')); print(d['value'], d.get('config2_literal',{}).get('value'), d.get('p50_image_latency_b1_ms'))"
done
echo done
