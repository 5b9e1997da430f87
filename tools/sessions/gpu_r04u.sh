#!/bin/bash
# (1) fused stage-1/2 attention with fragment-major weights (production) vs HEAD (base) and
# HEAD~1 (base1, before the window attention's buffer loads): per-op times of a 512-image
# encode, interleaved.  (2) decode chains: production vs the FFN fold GEMM on 32 x 64 tiles.
# (3) bench pipeline A/B.  (4) the GPU parity suite on production.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04u; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in base1 base production base production; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.,s2.,s3.,s4.wattn $(lib $L) > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|total" $O/ops_$L.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in production ffn64 production ffn64; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 2 --reps 2 $(lib $L) > $O/rows2_$L.log 2>&1 \
    || { echo "ROWS2 $L FAILED"; tail $O/rows2_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows2_$L.log | cut -c1-140
done
for L in base production s3fa base production s3fa; do
  timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; cut -c1-160 $O/bench_$L.json
done
echo done
