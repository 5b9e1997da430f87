#!/bin/bash
# Round-4 profile pass on the bench's shapes: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE in
# passes of their own) of one encode + 8 greedy steps at 512 and 640 images per call
# (tools/pmc_traffic.py -> profiles/pmc_traffic_bf16x3_b<B>.json), and rocprofv3
# --kernel-trace --stats of a short default bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04k; mkdir -p $O
for B in 512 640; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f$B -o run -- \
    python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_f$B.log 2>&1 || { echo "PMC F $B FAILED"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w$B -o run -- \
    python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_w$B.log 2>&1 || { echo "PMC W $B FAILED"; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_f$B/run_counter_collection.csv $O/pmc_w$B/run_counter_collection.csv \
    $O/pmc_traffic_bf16x3_b$B.json 8 $B || { echo "MAP $B FAILED"; exit 1; }
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-secondary > $O/prof_bench.log 2>&1 || { echo "ROCPROF FAILED"; tail $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $O/prof_bench/run_kernel_stats.csv 40 --no-load > $O/kstats_bench.txt
rm -f $O/prof_bench/run_kernel_trace.csv
head -12 $O/kstats_bench.txt
echo done
