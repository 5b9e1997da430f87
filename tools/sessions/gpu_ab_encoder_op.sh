#!/bin/bash
# Same-box A/B of an encoder-kernel variant build: bitwise stage maps (tests/probes/stage_diff.py),
# per-op HIP-event times (tools/op_times.py) and the bench pipeline (tools/pipeline_probe.py).
#   tools/sessions/gpu_ab_encoder_op.sh TAG LIB_A LIB_B FILTER     (e.g. FILTER=s3.)
mkdir -p gpurun_out
TAG=$1; A=$2; B=$3; F=${4:-s3.}
O=gpurun_out/ab_$TAG.log
: > $O
timeout -k 10 180 python tests/probes/stage_diff.py $A gpurun_out/sd_a.npz >> $O 2>&1 || exit 1
timeout -k 10 180 python tests/probes/stage_diff.py $B gpurun_out/sd_b.npz >> $O 2>&1 || exit 1
python -c "
import numpy as np
a=np.load('gpurun_out/sd_a.npz'); b=np.load('gpurun_out/sd_b.npz')
bad=[k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('stage maps bitwise equal' if not bad else 'DIFFER: %s' % bad)" >> $O
for lib in $A $B $A $B; do
  echo "== $lib" >> $O
  timeout -k 10 180 python tools/op_times.py --lib $lib --variants production --filter $F >> $O 2>&1 || exit 1
done
for lib in $A $B $A $B; do
  timeout -k 10 300 python -u tools/pipeline_probe.py --lib $lib --replicas 4 --modes encode,both --steps 16 >> $O 2>&1 || exit 1
done
grep -v amdgpu $O
