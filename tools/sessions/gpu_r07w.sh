#!/bin/bash
# Round 5 closing tree: rocprofv3 --kernel-trace --stats of a short bench (the kernel table
# behind DESIGN's per-kernel shares, after the stem / norm store staging).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07w; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-secondary > $O/prof_bench.log 2>&1 || { echo "ROCPROF FAILED"; tail $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $O/prof_bench/run_kernel_stats.csv 40 --no-load > $O/kstats_bench.txt
rm -f $O/prof_bench/run_kernel_trace.csv
head -14 $O/kstats_bench.txt
grep -E "stem16w|ln_group|split4" $O/kstats_bench.txt | cut -c1-150
grep '^{' $O/prof_bench.log | tail -1 > $O/bench_under_rocprof.json || true
echo done
