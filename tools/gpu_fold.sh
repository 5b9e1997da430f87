#!/bin/bash
# Folded decode step: GPU tests, then the headline bench with and without the fold (A/B).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-fold}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 120 ./tools/decode_kernels_bench > gpurun_out/deck_$TAG.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
MOCR_DEC_FOLD=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_off.json \
  2>> gpurun_out/bench_$TAG.err
echo done
