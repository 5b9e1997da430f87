#!/bin/bash
# GEMM microbenchmark over shapes: tools/sessions/gpu_gemm_sweep.sh TAG "M N K passes epi" ...
set -e
mkdir -p gpurun_out
TAG=$1
shift
for shape in "$@"; do
  echo "$shape | $(timeout -k 10 60 ./tools/gemm_bench $shape 20)" >> gpurun_out/gemm_$TAG.log
done
