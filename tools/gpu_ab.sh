#!/bin/bash
# GPU tests + GEMM A/B (run from the repo root on the GPU box); ring depths as args
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
for r in "$@"; do
  MOCR_GEMM_RING=$r timeout -k 10 180 python tools/gemm_ab.py --precision bf16x3 >> gpurun_out/ab.log 2>&1
  MOCR_GEMM_RING=$r timeout -k 10 180 python tools/gemm_ab.py --precision bf16 >> gpurun_out/ab.log 2>&1
done
