#!/bin/bash
# Phase-shape sweep of the 288-row GEMM (tools/gemm_bench force_kernel 10-17) on the
# stage-3 shapes: fc1 (288 x 256 tiles: PM x PN = 3x2 / 3x4 / 9x1 / 3x1), fc2 and proj
# (288 x 192: 3x3 / 9x1 / 3x1).  Ids 13-17 were a probe build's (gemm.hip launch_forced),
# removed after this sweep: profiles/r02/gemm_phase_sweep.log.
mkdir -p gpurun_out
O=gpurun_out/gemm_phase_sweep.log
: > $O
run() { echo "$* | $(timeout -k 5 60 ./tools/gemm_bench "$@")" >> $O || exit 1; }
for rep in 1 2; do
  for k in 10 13 14 15; do run 36864 1536 384 3 1 30 1 $k; done
  for k in 11 16 17; do run 36864 384 1536 3 2 30 1 $k; done
  for k in 11 16 17; do run 36864 384 384 3 2 30 1 $k; done
done
cat $O
