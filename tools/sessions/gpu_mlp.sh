#!/bin/bash
# Fused MLP: GPU tests, bench, LDS-conflict / instruction counters of one encode.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_$TAG -o run -- python3 tools/profile_encoder.py > gpurun_out/pmc_$TAG.log 2>&1
echo done
