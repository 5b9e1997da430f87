#!/bin/bash
# Round 5 A/B of two prologue-hiding variants against production:
#  - s3pf: stage-3 attention on persistent workgroups, the next window's X rows DMA'd into
#    LDS while the current window's attention runs (-DMOCR_S3_PF=1);
#  - nh: merge 1 (lngemm384, N = 192) on persistent workgroups holding half of W resident
#    in LDS (-DMOCR_MERGE1_NH=1).
# Per-op times of a 512-image encode, the encoder parity tests on each variant, the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06u; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
for L in production s3pf nh production s3pf nh; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 2 --variants production --filter s3.attn,merge1 $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|merge|total" $O/ops_$L.log
done
cp $P /tmp/prod_lib.so
for V in s3pf nh; do
  cp handwritten-math-ocr-api_amd/lib_var/$V/libmathocr.so $P
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
    -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched" > $O/tests_$V.log 2>&1 \
    || { echo "TESTS $V FAILED"; tail -30 $O/tests_$V.log; cp /tmp/prod_lib.so $P; exit 1; }
  echo "tests $V: $(tail -1 $O/tests_$V.log)"
  cp /tmp/prod_lib.so $P
done
for L in production s3pf nh production s3pf nh; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
