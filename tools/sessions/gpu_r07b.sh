#!/bin/bash
# Round 5: VALU trims in the fused encoder kernels vs HEAD (lib_var/base):
#  - window attention: softmax in base 2 (log2 e folded into q's scale and a second bias
#    table), the bias tile as the S MFMAs' accumulator input;
#  - fused MLPs: 2 x GELU against W2 / 2 chunk images (bitwise the same outputs).
# Bitwise check of the MLP change (unfused attention, so only the MLP change differs),
# per-op times, the parity tests, the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07b; mkdir -p $O
B=handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_base.npy --lib $B --variant unfused_attn > $O/mem.log 2>&1 || { echo "MEM BASE FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_new.npy --variant unfused_attn >> $O/mem.log 2>&1 || { echo "MEM NEW FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_base.npy'); b=np.load('$O/mem_new.npy'); print('mlp change bitwise equal (unfused attention):', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in base production base production; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.,s2.,s3. $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|total" $O/ops_$L.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_conditioning.py -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for L in base production base production; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
