#!/bin/bash
# Round 5 timing probe: the int16 self-attention cache without its per-key scale loads
# (lib_var/scprobe, wrong results) vs production: one 512-row decode chain, rocprof stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06w; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production scprobe production scprobe; do
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512 --chains 1 --reps 3 $(lib $L) > $O/chains_$L.log 2>&1 \
    || { echo "CHAINS $L FAILED"; tail $O/chains_$L.log; exit 1; }
  echo "== chains $L $(grep rows_per_s $O/chains_$L.log | tail -1)"
done
for L in production scprobe; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$L -o run -- \
    python3 tools/decode_chain_probe.py --rows 512 --chains 1 --reps 1 $(lib $L) > $O/prof_$L.log 2>&1 || { echo "PROF $L FAILED"; exit 1; }
  python3 tools/kstats.py $O/prof_$L/run_kernel_stats.csv 14 --no-load > $O/kstats_$L.txt
  rm -f $O/prof_$L/run_kernel_trace.csv
  echo "== kstats $L"; grep "dec_foldattn_kernel<true" $O/kstats_$L.txt | head -6
done
echo done
