#!/bin/bash
# Config 4 (beam 4, B = 32, 256 tokens) regression: the round-2 tree (tmp_r02, commit
# 42abab6) vs the current tree on one box -- bench A/B, then kernel traces of a short
# bench of each for GPU occupancy (tools/trace_busy.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04i; mkdir -p $O
for rep in 1 2; do
  (cd tmp_r02 && timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 24 2>/dev/null | cut -c1-160) || exit 1
  timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --no-secondary --steps 24 2>/dev/null | cut -c1-160 || exit 1
done
(cd tmp_r02 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ../$O/r02 -o run -- python3 bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 8 --warmup 4 --no-isolated > ../$O/r02.log 2>&1) || { echo r02 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cur -o run -- python3 bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --no-secondary --steps 8 --warmup 4 --no-isolated > $O/cur.log 2>&1 || { echo cur failed; exit 1; }
echo "== r02"; python3 tools/trace_busy.py $O/r02/run_kernel_trace.csv beam_select
echo "== cur"; python3 tools/trace_busy.py $O/cur/run_kernel_trace.csv beam_select
echo done
