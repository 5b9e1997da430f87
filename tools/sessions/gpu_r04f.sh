#!/bin/bash
# Pipelined bench, second sweep: the driver's 20-step form at other chain x replica
# shapes, and 64 steps at 8 x 64 with 2 / 4 replicas and 16 x 64 with 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04f; mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --no-isolated "$@" > $O/b_$tag.json 2> $O/b_$tag.err \
    || { echo "BENCH $tag FAILED"; tail -5 $O/b_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b_$tag.json')); c=d['config']; print('$tag', round(d['value']), 'G', c['batches_per_chain'], 'R', c['replicas_per_gpu'], 'steps', d['steps'], 'p50', round(d['p50_image_latency_ms']))"
}
run s20g5r2 --steps 20 --warmup 5 --chain-batches 5 --replicas 2
run s20g10r2 --steps 20 --warmup 20 --chain-batches 10 --replicas 2
run s20g5r4 --steps 20 --warmup 20 --chain-batches 5 --replicas 4
run s20g4r5 --steps 20 --warmup 20 --chain-batches 4 --replicas 5
run s64g8r2 --steps 64 --warmup 16 --chain-batches 8 --replicas 2
run s64g8r4 --steps 64 --warmup 32 --chain-batches 8 --replicas 4
run s64g16r2 --steps 64 --warmup 32 --chain-batches 16 --replicas 2
echo done
