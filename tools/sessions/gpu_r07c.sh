#!/bin/bash
# Round 5: fused MLPs with b1 as GEMM 1's accumulator input (production build of the tree)
# and, on top, the stage-1 MLP held to 168 registers for three waves per SIMD
# (lib_var/occ3, 144 B of scratch), vs HEAD (lib_var/base). Per-op times, parity, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07c; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in base production occ3 base production occ3; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.mlp,s2.mlp,s3.mlp $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "mlp|total" $O/ops_$L.log
done
P=handwritten-math-ocr-api_amd/lib/libmathocr.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_conditioning.py -x -q --timeout 300 --timeout-method thread \
  > $O/tests_production.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests_production.log; exit 1; }
echo "tests production: $(tail -1 $O/tests_production.log)"
cp $P /tmp/prod_lib.so; cp handwritten-math-ocr-api_amd/lib_var/occ3/libmathocr.so $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "encoder_stages or memory_matches" \
  > $O/tests_occ3.log 2>&1 || { echo "TESTS OCC3 FAILED"; tail -30 $O/tests_occ3.log; cp /tmp/prod_lib.so $P; exit 1; }
echo "tests occ3: $(tail -1 $O/tests_occ3.log)"; cp /tmp/prod_lib.so $P
for L in base production occ3 base production occ3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
