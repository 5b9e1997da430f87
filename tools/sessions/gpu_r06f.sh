#!/bin/bash
# Round 5: the stage-1/2 fused attention with two windows per workgroup (lib_var/s1w2:
# stage 1; lib_var/s12w2: stages 1 and 2), the stage-1 MLP on 4-wave workgroups with
# 32-unit chunks (lib_var/mlp4), and all three (lib_var/comb) vs production: per-op times
# of a 512-image encode, the parity of the encoder tests on each, then the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06f; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
for L in production s1w2 s12w2 mlp4 comb production s1w2 s12w2 mlp4 comb; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 2 --variants production --filter s1.,s2. $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|total" $O/ops_$L.log
done
cp $P /tmp/prod_lib.so
for L in s1w2 s12w2 mlp4 comb; do
  cp handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so $P
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "encoder_stages or memory_matches or greedy_ids_match or bf16_encoder_modes" > $O/tests_$L.log 2>&1 \
    || { echo "TESTS $L FAILED"; tail -30 $O/tests_$L.log; cp /tmp/prod_lib.so $P; exit 1; }
  echo "tests $L: $(tail -1 $O/tests_$L.log)"
done
cp /tmp/prod_lib.so $P
for L in production comb production comb; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
