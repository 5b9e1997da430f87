#!/bin/bash
# Decode step vs rows per chain (does a kernel's second round show up?): chain probe at
# 256..512 rows, rocprofv3 kernel stats of one chain at 320 and 512 rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 192,256,288,320,384,448,512 --chains 1 --reps 2 > $O/rows.log 2>&1 \
  || { echo "ROWS FAILED"; tail $O/rows.log; exit 1; }
grep rows_per_s $O/rows.log
for R in 320 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec$R -o run -- \
    python3 tools/decode_chain_probe.py --rows $R --chains 1 --reps 1 > $O/dec$R.log 2>&1 || { echo "PROF $R FAILED"; exit 1; }
done
echo done
