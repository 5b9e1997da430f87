#!/bin/bash
# Same-box A/B of two libmathocr.so builds on the bench pipeline (tools/pipeline_probe.py):
#   tools/sessions/gpu_ab_pipeline.sh TAG LIB_A LIB_B   (alternating A B A B, encode-only and both)
mkdir -p gpurun_out
O=gpurun_out/ab_$1.log
: > $O
for lib in $2 $3 $2 $3; do
  timeout -k 10 300 python -u tools/pipeline_probe.py --lib $lib --replicas 4 --modes encode,both --steps 16 >> $O 2>&1 || exit 1
done
grep -v amdgpu $O
