#!/bin/bash
# Round 5: stem16 grid sized to its occupancy (3 waves/SIMD: 768 workgroups = one resident
# round; 1536 = two) vs production 1024 (a second, quarter-full round). Stem time, bench.
# (Each token is independent of the grid, so the memory is bitwise the same by construction.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07k; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production stem768 stem1536 production stem768 stem1536; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter stem $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "stem" $O/ops_$L.log
done
for L in production stem768 stem1536 production stem768 stem1536; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
