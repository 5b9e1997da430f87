#!/bin/bash
# Round 5: vectorised bf16 hi/lo split (split4_bf16_kernel: float4 in, 8-B stores) vs HEAD's
# scalar split (lib_var/base). Bitwise memory + 24 decode steps' logits and ids, split time;
# the stem's prefetch depth 2 (lib_var/stemd2, bitwise memory + stem time); then the final
# tree's whole GPU suite, smoke and both bench forms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07o; mkdir -p $O
B=handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy --decode 24 > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_base.npy --decode 24 --lib $B >> $O/mem.log 2>&1 || { echo "MEM BASE FAILED"; tail $O/mem.log; exit 1; }
python - <<PY
import numpy as np
for s in ("", "_logits", "_ids"):
    a = np.load("$O/mem_prod%s.npy" % s); b = np.load("$O/mem_base%s.npy" % s)
    print("split4 vs base%s bitwise equal:" % (s or "_memory"), bool((a.view(np.uint32) == b.view(np.uint32)).all()), a.shape)
PY
timeout -k 10 200 python tools/mem_dump.py $O/mem_d2.npy --lib handwritten-math-ocr-api_amd/lib_var/stemd2/libmathocr.so >> $O/mem.log 2>&1 || { echo "MEM D2 FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_d2.npy'); print('stemd2 memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
for L in production base stemd2 production base stemd2; do
  X=""; [ $L != production ] && X="--lib handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so"
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter split,stem $X \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "split|stem" $O/ops_$L.log
done
rm -f $O/*.npy
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "BENCH FAILED"; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config2_literal',{}).get('value'))"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "BENCH DRIVER FAILED"; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver', d['value'], d['ms_per_step'])"
echo done
