#!/bin/bash
# Round 5: stem16w prefetch depth (production: 1 sweep ahead) vs 2 sweeps (lib_var/stemd2) and
# the old stem16 (lib_var/stemd0). Bitwise memory of depth 2, stem time, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07n; mkdir -p $O
timeout -k 10 200 python tools/mem_dump.py $O/mem_prod.npy > $O/mem.log 2>&1 || { echo "MEM PROD FAILED"; tail $O/mem.log; exit 1; }
timeout -k 10 200 python tools/mem_dump.py $O/mem_var.npy --lib handwritten-math-ocr-api_amd/lib_var/stemd2/libmathocr.so >> $O/mem.log 2>&1 || { echo "MEM VAR FAILED"; tail $O/mem.log; exit 1; }
python -c "import numpy as np; a=np.load('$O/mem_prod.npy'); b=np.load('$O/mem_var.npy'); print('stemd2 memory bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()), a.shape)"
rm -f $O/*.npy
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production stemd2 stemd0 production stemd2 stemd0; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter stem $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "stem" $O/ops_$L.log
done
for L in production stemd2 production stemd2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
