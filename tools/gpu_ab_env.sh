#!/bin/bash
# GPU tests, then tools/gemm_ab.py (bf16x3 and bf16) once per environment setting given
# as arguments, e.g.  bash tools/gpu_ab_env.sh MOCR_GEMM_BIG_MIN=0 MOCR_GEMM_BIG_MIN=384
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
for kv in "$@"; do
  env "$kv" timeout -k 10 180 python tools/gemm_ab.py --precision bf16x3 | sed "s/\"ring\": \"[^\"]*\"/\"ring\": \"$kv\"/" >> gpurun_out/ab.log
  env "$kv" timeout -k 10 180 python tools/gemm_ab.py --precision bf16 | sed "s/\"ring\": \"[^\"]*\"/\"ring\": \"$kv\"/" >> gpurun_out/ab.log
done
