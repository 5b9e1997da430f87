#!/bin/bash
# Round 5: stage 3 on swin_attn_kernel<384> (norm1 + qkv + W-MSA + proj + residual in one kernel)
# (lib_var/s3fp) vs production:
# per-op times of a 512-image encode, the encoder parity tests on the variant, the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06q; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
for L in production s3fp production s3fp; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 2 --variants production --filter s1.,s2.,s3. $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|proj|total" $O/ops_$L.log
done
cp $P /tmp/prod_lib.so
cp handwritten-math-ocr-api_amd/lib_var/s3fp/libmathocr.so $P
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes or as_benched_b256" > $O/tests_s3fp.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests_s3fp.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests s3fp: $(tail -1 $O/tests_s3fp.log)"
cp /tmp/prod_lib.so $P
for L in production s3fp production s3fp; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
