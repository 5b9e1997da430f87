#!/bin/bash
# rocprofv3 kernel stats of decode-only pipelines at 1 and 3 replicas
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec$r -o run -- python3 tools/pipeline_probe.py --replicas $r --steps 6 --modes decode > gpurun_out/prof_dec$r.log 2>&1
done
