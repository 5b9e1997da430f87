#!/bin/bash
# Replica-count sweep of the bench pipeline on the current build (both halves, 24 batches):
#   tools/sessions/gpu_replica_sweep.sh TAG
mkdir -p gpurun_out
O=gpurun_out/replicas_$1.log
: > $O
for rep in 1 2; do
  for r in 4 5 6; do
    timeout -k 10 300 python -u tools/pipeline_probe.py --replicas $r --modes both --steps 24 >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu $O
