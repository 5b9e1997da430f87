#!/bin/bash
# Same-box A/B of two libmathocr.so builds on decode-only and full-pipeline capacity
# (tools/pipeline_probe.py, 4 replicas; decode-only also at 1 replica), alternating A B A B.
#   tools/sessions/gpu_ab_decode.sh TAG LIB_A LIB_B
mkdir -p gpurun_out
O=gpurun_out/abd_$1.log
: > $O
for lib in $2 $3 $2 $3; do
  timeout -k 10 200 python -u tools/pipeline_probe.py --lib $lib --replicas 1 --modes decode --steps 4 >> $O 2>&1 || exit 1
  timeout -k 10 300 python -u tools/pipeline_probe.py --lib $lib --replicas 4 --modes decode,both --steps 16 >> $O 2>&1 || exit 1
done
grep -v amdgpu $O
