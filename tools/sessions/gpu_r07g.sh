#!/bin/bash
# Round 5: int16 K/V rows kept packed until the attention loops convert them (cross-attention
# 81 -> 71 VGPRs: 5 -> 7 waves per SIMD) vs HEAD (lib_var/base). Bitwise decode check,
# decode chains, the decode parity tests, the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07g; mkdir -p $O
B=handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/base.npy --lib $B --batch 64 --decode 40 > $O/dump.log 2>&1 || { echo "DUMP BASE FAILED"; tail $O/dump.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/new.npy --batch 64 --decode 40 >> $O/dump.log 2>&1 || { echo "DUMP NEW FAILED"; tail $O/dump.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/base_logits.npy'); b=np.load('$O/new_logits.npy'); print('decode logits bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape, 'ids equal:', bool((np.load('$O/base_ids.npy')==np.load('$O/new_ids.npy')).all()))"
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in base production base production; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512 --chains 1,2 --reps 2 $(lib $L) > $O/chains_$L.log 2>&1 \
    || { echo "CHAINS $L FAILED"; tail $O/chains_$L.log; exit 1; }
  echo "== chains $L"; grep rows_per_s $O/chains_$L.log | tail -2 | cut -c1-130
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_conditioning.py tests/test_gpu_beam.py -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for L in base production base production; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
