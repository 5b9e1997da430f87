#!/bin/bash
# Round 5: the greedy decode step alone under rocprofv3 (one 512-row chain and one 640-row
# chain, 128 steps each): per-kernel durations of the step, to set beside the bench's
# HIP-event step time (roofline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06k; mkdir -p $O
for R in 512 640; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dec$R -o run -- \
    python3 tools/decode_chain_probe.py --rows $R --chains 1 --reps 1 > $O/dec$R.log 2>&1 || { echo "PROF $R FAILED"; tail $O/dec$R.log; exit 1; }
  python3 tools/kstats.py $O/prof_dec$R/run_kernel_stats.csv 30 --no-load > $O/kstats_dec$R.txt
  rm -f $O/prof_dec$R/run_kernel_trace.csv
  grep rows_per_s $O/dec$R.log | cut -c1-160
  python3 -c "
import csv
rows = list(csv.DictReader(open('$O/prof_dec$R/run_kernel_stats.csv')))
dec = [r for r in rows if any(k in r['Name'] for k in ('dec_foldattn', 'foldwide', 'dec_argmax'))]
tot = sum(float(r['TotalDurationNs']) for r in dec)
print('decode kernels: %d launches, %.1f us of kernel time per step (2 decodes x 128 steps)' % (sum(int(r['Calls']) for r in dec), tot / 256 / 1e3))
" | tee $O/step_sum_dec$R.txt
  head -12 $O/kstats_dec$R.txt
done
echo done
