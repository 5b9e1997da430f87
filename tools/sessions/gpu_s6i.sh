#!/bin/bash
# Round 6: phase clocks of the decode kernels at the bench's 640-row chain (tools/fold_ts,
# tools/attn_ts against lib_var/ts, built with -DMOCR_FOLD_TS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s6i; mkdir -p $O
for a in "256 256" "512 768" "256 0"; do
  echo "== fold_ts 640 $a" >> $O/phase.txt
  timeout -k 10 60 tools/fold_ts 640 $a >> $O/phase.txt 2>&1 || { echo "FOLD_TS $a FAILED"; tail $O/phase.txt; exit 1; }
done
for a in "cross 640" "self 640 16" "self 640 120"; do
  echo "== attn_ts $a" >> $O/phase.txt
  timeout -k 10 60 tools/attn_ts $a >> $O/phase.txt 2>&1 || { echo "ATTN_TS $a FAILED"; tail $O/phase.txt; exit 1; }
done
cat $O/phase.txt
