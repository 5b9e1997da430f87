#!/bin/bash
# Round 5 final tree: per-op HIP-event times of a 512-image encode (every op, one replica
# alone), for DESIGN's current per-op table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production > $O/ops_all.log 2>&1 || { echo "OPS FAILED"; tail $O/ops_all.log; exit 1; }
cat $O/ops_all.log | grep -v amdgpu.ids
echo done
