#!/bin/bash
# (1) window attention: buffer-load addressing + padded key tile skip (production) vs HEAD
# (base); swin_attn_kernel probes 6 (half the weight-fragment loads) and 7 (one bias tile
# per window): per-op times of a 512-image encode.  (2) decode chains: greedy logits
# without stores (production) vs HEAD, and the FFN fold GEMM on 32 x 64 tiles (ffn64).
# (3) bench pipeline A/B.  (4) the GPU parity suite on production.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04t; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in base production wp6 wp7 base production; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.attn,s2.attn,s3.wattn,s4.wattn $(lib $L) > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn" $O/ops_$L.log
done
for L in base production ffn64 base production ffn64; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 1 --reps 2 $(lib $L) > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 2 --reps 2 $(lib $L) > $O/rows2_$L.log 2>&1 \
    || { echo "ROWS2 $L FAILED"; tail $O/rows2_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log $O/rows2_$L.log | cut -c1-140
done
# (3) the bench pipeline (8 x 64 images per call, 2 replicas, 32 timed batches):
# production vs HEAD vs the fused stage-3 attention at every batch (s3fa) vs ffn64
for L in base production s3fa ffn64 production s3fa; do
  timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; cut -c1-160 $O/bench_$L.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
