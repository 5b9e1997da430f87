#!/bin/bash
# GPU tests, then decode-only capacity with / without the fused projection+attention,
# then replica counts with 8 HW queues (run from the repo root on the GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
for f in 0 1; do for r in 1 3; do
  MOCR_DEC_FUSED=$f timeout -k 10 300 python tools/pipeline_probe.py --replicas $r --steps 12 --modes decode > gpurun_out/dec_ab_$f_$r.json 2>>gpurun_out/dec_ab.err
  echo "fused=$f $(cat gpurun_out/dec_ab_$f_$r.json)" >> gpurun_out/dec_ab.log
done; done
for r in 4 6 8; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/pipeline_probe.py --replicas $r --steps 16 >> gpurun_out/probe_q.json 2>>gpurun_out/dec_ab.err
done
