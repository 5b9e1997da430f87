#!/bin/bash
# GEMM dispatch A/B on the encoder shapes: tools/sessions/gpu_gemm_ab.sh TAG
# (gemm_bench: kernel -1 = the dispatch before the 288-row tiles, 0 = the current dispatch)
mkdir -p gpurun_out
TAG=${1:-ab}
O=gpurun_out/gemm_ab_$TAG.log
: > $O
run() { echo "$* | $(timeout -k 5 60 ./tools/gemm_bench "$@")" >> $O || exit 1; }
for rep in 1 2; do
for k in -1 0; do run 36864 1536 384 3 1 30 1 $k; done          # s3.fc1 (GELU, bf16 planes out)
for k in -1 0; do run 36864 384 1536 3 2 30 1 $k; done          # s3.fc2 (residual add)
for k in -1 0; do run 36864 384 384 3 2 30 1 $k; done           # s3.proj-shaped
for k in -1 0; do run 9216 3072 768 3 1 30 1 $k; done           # s4.fc1
for k in -1 0; do run 9216 768 3072 3 2 30 1 $k; done           # s4.fc2
for k in -1 0; do run 147456 192 384 3 0 30 1 $k; done          # merge1
for k in -1 0; do run 36864 384 768 3 0 30 1 $k; done           # merge2
for k in -1 0; do run 9216 768 1536 3 0 30 1 $k; done           # merge3
for k in -1 0; do run 9216 4096 256 3 0 30 1 $k; done           # crosskv
done
cat $O
