#!/bin/bash
# The fused stage-3 no-proj attention at every batch (s3fa), now on fragment-major W_qkv,
# vs production (lngemm384 + window attention above 128 images): per-op times of a
# 512-image encode and the bench pipeline, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04x; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production s3fa production s3fa; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s3. $(lib $L) > $O/ops512_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops512_$L.log; exit 1; }
  echo "== $L"; grep -E "s3|total" $O/ops512_$L.log
done
for L in production s3fa production s3fa; do
  timeout -k 10 400 python -u bench.py --steps 32 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench_$L.json 2> $O/bench_$L.err || { echo "BENCH $L FAILED"; tail $O/bench_$L.err; exit 1; }
  echo "== bench $L"; python -c "import json; d=json.load(open('$O/bench_$L.json')); print(d['value'])"
done
echo done
