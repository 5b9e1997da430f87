#!/bin/bash
# GEMM variant matrix on encoder shapes (tools/gemm_bench) + GPU tests with K-concat on
set -e
mkdir -p gpurun_out
MOCR_GEMM_KCAT=1 MOCR_GEMM_STAGES=3 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_kcat.log 2>&1
B=./tools/gemm_bench
for v in "MOCR_GEMM_BIG_MIN=0" "MOCR_GEMM_BIG_MIN=384" "MOCR_GEMM_KCAT=1 MOCR_GEMM_STAGES=2" "MOCR_GEMM_KCAT=1 MOCR_GEMM_STAGES=3" \
         "MOCR_GEMM_KCAT=1 MOCR_GEMM_STAGES=4" "MOCR_GEMM_KCAT=1 MOCR_GEMM_KBIG=1 MOCR_GEMM_STAGES=2" \
         "MOCR_GEMM_KCAT=1 MOCR_GEMM_KBIG=1 MOCR_GEMM_STAGES=3"; do
  for shape in "36864 1536 384 3 1" "36864 384 1536 3 2" "9216 3072 768 3 1" "614656 384 96 3 1" "36864 1152 384 3 0"; do
    echo "$v | $(env $v timeout -k 10 60 $B $shape 20)" >> gpurun_out/gemm_matrix.log
  done
done
