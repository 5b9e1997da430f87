#!/bin/bash
# GPU tests, then the headline bench under environment variants: tools/gpu_ab.sh TAG "ENV=.." ...
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$TAG.log 2>&1
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err
  echo "$i $v" >> gpurun_out/bench_${TAG}_index.txt
done
echo done
