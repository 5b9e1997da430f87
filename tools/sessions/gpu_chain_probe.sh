#!/bin/bash
# Decode capacity by rows per chain x chains, and rocprofv3 kernel stats of one 64-row and
# one 256-row chain (tools/decode_chain_probe.py).  Usage: tools/sessions/gpu_chain_probe.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-chain}
mkdir -p $O
timeout -k 10 400 python3 -u tools/decode_chain_probe.py > $O/chain_probe.log 2>&1 || { echo "PROBE FAILED"; tail -20 $O/chain_probe.log; exit 1; }
cat $O/chain_probe.log
for R in 64 256; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$R -o run -- \
    python3 tools/decode_chain_probe.py --rows $R --chains 1 --reps 1 > $O/prof$R.log 2>&1 || { echo "PROF $R FAILED"; tail -20 $O/prof$R.log; exit 1; }
  rm -f $O/prof$R/run_kernel_trace.csv
done
echo done
