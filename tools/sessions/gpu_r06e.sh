#!/bin/bash
# Round 5: beam search on the folded step -- beam tests (folded + unfolded), config 4
# (beam 4, B = 32, 256 tokens) bench on both paths, then the greedy suite's decode tests
# (the fold attention kernel changed: mem_div, slot tables).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_full.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "beam or config4" > $O/tests_beam.log 2>&1 || { echo "BEAM TESTS FAILED"; tail -60 $O/tests_beam.log; exit 1; }
tail -1 $O/tests_beam.log
for V in folded unfolded; do
  X=""; [ $V = unfolded ] && X="--variant beam_unfolded"
  timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --steps 24 --warmup 4 --no-cpu-baseline $X \
    > $O/bench_c4_$V.json 2> $O/bench_c4_$V.err || { echo "BENCH C4 $V FAILED"; tail $O/bench_c4_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_c4_$V.json')); print('C4 $V', d['value'], d['ms_per_step'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests_all.log 2>&1 || { echo "SUITE FAILED"; tail -60 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
echo done
