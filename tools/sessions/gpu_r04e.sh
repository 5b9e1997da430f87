#!/bin/bash
# Pipelined bench by chain length x replicas (same box): the driver's 20-step form, and
# 32 batches at 8 x 64 / 4 x 64 / 5 x 64.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04e; mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --no-isolated "$@" > $O/b_$tag.json 2> $O/b_$tag.err \
    || { echo "BENCH $tag FAILED"; tail -5 $O/b_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b_$tag.json')); c=d['config']; print('$tag', round(d['value']), 'G', c['batches_per_chain'], 'R', c['replicas_per_gpu'], 'steps', d['steps'], 'p50', round(d['p50_image_latency_ms']))"
}
run s40g4r2 --steps 40 --warmup 8 --chain-batches 4 --replicas 2
run s40g5r2 --steps 40 --warmup 10 --chain-batches 5 --replicas 2
run s32g8r2 --steps 32 --warmup 16 --chain-batches 8 --replicas 2
run s48g8r3 --steps 48 --warmup 24 --chain-batches 8 --replicas 3
run s48g4r3 --steps 48 --warmup 12 --chain-batches 4 --replicas 3
run s36g6r2 --steps 36 --warmup 12 --chain-batches 6 --replicas 2
echo done
