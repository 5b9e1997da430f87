#!/bin/bash
# Baseline pass on the GPU box (repo root): GPU tests, GEMM / decode microbenchmarks,
# headline bench, rocprofv3 kernel stats of a short bench.  Each GPU step has its own
# time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-base}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$TAG.log 2>&1
G=./tools/gemm_bench
for shape in "36864 1536 384 3 1" "36864 1536 384 3 0" "36864 1536 768 3 0" "36864 1536 1536 3 0" \
             "18432 1536 384 3 1" "9216 3072 768 3 1" "36864 384 1536 3 2"; do
  echo "$shape | $(timeout -k 10 60 $G $shape 20)" >> gpurun_out/gemm_$TAG.log
done
timeout -k 10 120 ./tools/decode_kernels_bench > gpurun_out/deck_$TAG.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo done
