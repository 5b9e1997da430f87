#!/bin/bash
# Round 5: the multi-rank bench path on the one-GPU box (two ranks share cuda:0, gather over
# gloo; the driver's N > 1 command form), and bench.py --gpus 2 without a launcher.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 8 --warmup 4 > $O/bench_n2_driver.json 2> $O/bench_n2_driver.err || { echo "N2 DRIVER FAILED"; tail -20 $O/bench_n2_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_driver.json')); print('n2 driver', d['value'], d['n_gpus'], d.get('rccl_ranks'), d.get('rank_elapsed_s'), d['config'].get('gather'))"
timeout -k 10 600 python bench.py --gpus 2 --steps 8 --warmup 4 > $O/bench_n2_self.json 2> $O/bench_n2_self.err || { echo "N2 SELF FAILED"; tail -20 $O/bench_n2_self.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_self.json')); print('n2 self', d['value'], d['n_gpus'], d.get('rccl_ranks'), d['config'].get('gather'))"
echo done
