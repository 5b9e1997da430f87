#!/bin/bash
# Forced-kernel sweep of the stage-4 GEMM shapes (M = 9216 at B = 64, 384²): tools/gemm_bench
# force_kernel 0 (dispatch), 3 tile16, 10/11/12 288 x 256/192/128 (the shapes where they all fit).
mkdir -p gpurun_out
O=gpurun_out/gemm_s4_sweep.log
: > $O
for rep in 1 2; do
for shape in "9216 2304 768 3 0" "9216 768 768 3 2"; do
  for k in 0 3 10 11 12; do
    echo "$shape k$k | $(timeout -k 5 60 ./tools/gemm_bench $shape 30 1 $k 2>&1 | tail -1)" >> $O || exit 1
  done
done
done
cat $O
