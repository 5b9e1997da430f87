#!/bin/bash
# staggered 256x256 GEMM vs the ring kernels: timing + output checksums, then GPU tests
set -e
mkdir -p gpurun_out
B=./tools/gemm_bench
for shape in "36864 1536 384 3 1" "9216 3072 768 3 1" "147456 768 192 3 1" "9216 4096 256 3 0" "9216 768 3072 3 2" \
             "36864 1536 384 1 1" "9216 3072 768 1 1" "9216 4096 256 1 0"; do
  for v in "MOCR_GEMM_BIG_MIN=0" "MOCR_GEMM_BIG_MIN=384" "MOCR_GEMM_STAG_MIN=1"; do
    echo "$v | $(env $v timeout -k 10 60 $B $shape 20)" >> gpurun_out/stag.log
  done
done
MOCR_GEMM_STAG_MIN=1 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_stag.log 2>&1
