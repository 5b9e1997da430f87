#!/bin/bash
# Decode-kernel microbenchmark under environment variants: tools/sessions/gpu_deck.sh TAG "ENV=.." ...
set -e
mkdir -p gpurun_out
TAG=$1
shift
for v in "$@"; do
  echo "== $v" >> gpurun_out/deck_$TAG.log
  env $v timeout -k 10 120 ./tools/decode_kernels_bench >> gpurun_out/deck_$TAG.log 2>&1
done
