#!/bin/bash
# Round 5 timing probe: every row's cross-attention reads memory row 0's K/V (L2-resident;
# lib_var/xprobe, wrong results) vs production -- what the int16 cross K/V stream costs the
# decode alone and the pipelined bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06t; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production xprobe; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512 --chains 1,2 --reps 2 $(lib $L) > $O/chains_$L.log 2>&1 \
    || { echo "CHAINS $L FAILED"; tail $O/chains_$L.log; exit 1; }
  echo "== chains $L"; grep -E "rows" $O/chains_$L.log | tail -4
done
for L in production xprobe production xprobe; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-isolated --no-secondary --no-cpu-baseline $(lib $L) \
    > $O/bench20_$L.json 2> $O/bench20_$L.err || { echo "BENCH $L FAILED"; tail $O/bench20_$L.err; exit 1; }
  echo "== bench20 $L $(python -c "import json; print(json.load(open('$O/bench20_$L.json'))['value'])")"
done
echo done
