#!/bin/bash
# rocprofv3 kernel stats of one decode chain per row count.  Usage: tools/sessions/gpu_chain_prof.sh TAG ROWS...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-cp}
shift
mkdir -p $O
for R in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$R -o run -- \
    python3 tools/decode_chain_probe.py --rows $R --chains 1 --reps 1 > $O/prof$R.log 2>&1 || { echo "PROF $R FAILED"; tail -20 $O/prof$R.log; exit 1; }
  rm -f $O/prof$R/run_kernel_trace.csv
  python3 tools/kstats.py $O/prof$R/run_kernel_stats.csv 14
done
