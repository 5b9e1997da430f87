#!/bin/bash
# Encode-only / decode-only / both capacity vs replicas (tools/pipeline_probe.py): tools/sessions/gpu_probe.sh TAG MODES R...
set -e
mkdir -p gpurun_out
TAG=$1
MODES=$2
shift 2
for r in "$@"; do
  echo "== replicas $r" >> gpurun_out/probe_$TAG.log
  timeout -k 10 300 python tools/pipeline_probe.py --replicas $r --steps 16 --modes $MODES >> gpurun_out/probe_$TAG.log 2>&1
done
