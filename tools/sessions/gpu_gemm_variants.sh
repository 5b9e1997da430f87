#!/bin/bash
# Same GEMM shapes through gemm_bench binaries linked against variant libraries:
# tools/sessions/gpu_gemm_variants.sh TAG VARIANT...   (tools/gemm_bench_VARIANT; "base" = tools/gemm_bench)
mkdir -p gpurun_out
TAG=$1; shift
O=gpurun_out/gemm_var_$TAG.log
: > $O
run() { local b=$1; shift; echo "$b $* | $(timeout -k 5 60 $b "$@")" >> $O || exit 1; }
for rep in 1 2; do
  for v in "$@"; do
    b=./tools/gemm_bench_$v; [ "$v" = base ] && b=./tools/gemm_bench
    run $b 36864 1536 384 3 1 30 1      # s3.fc1
    run $b 36864 384 1536 3 2 30 1      # s3.fc2
    run $b 36864 384 384 3 2 30 1       # s3.proj
  done
done
cat $O
