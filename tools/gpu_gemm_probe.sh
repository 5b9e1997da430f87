#!/bin/bash
# GEMM microbenchmarks + SQ counters on the s3.fc1 shape, decode kernel timings, GPU tests
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
B=./tools/gemm_bench
for v in "MOCR_GEMM_BIG_MIN=0" "MOCR_GEMM_BIG_MIN=384"; do
  for shape in "36864 1536 384 3 1" "36864 384 1536 3 2" "9216 3072 768 3 1" "614656 384 96 3 1"; do
    echo "$v $(env $v timeout -k 10 60 $B $shape 20)" >> gpurun_out/gemm_probe.log
  done
done
timeout -k 10 120 ./tools/decode_kernels_bench > gpurun_out/dec_kernels.log 2>&1
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true
for v in "MOCR_GEMM_BIG_MIN=0" "MOCR_GEMM_BIG_MIN=384"; do
  tag=$(echo $v | tr '=' '_')
  export $v
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_gemm_$tag -o a -- $B 36864 1536 384 3 1 5 > gpurun_out/pmc_gemm_$tag.log 2>&1 || true
  timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_gemm2_$tag -o a -- $B 36864 1536 384 3 1 5 >> gpurun_out/pmc_gemm_$tag.log 2>&1 || true
done
