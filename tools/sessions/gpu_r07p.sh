#!/bin/bash
# Round 5 final measurement pass (stem16w, vectorised split, stage-1/2 MLP DMA): rocprofv3 --kernel-trace --stats of a short
# bench (the roofline's kernels), PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of one
# encode + 8 greedy steps at 512 and 640 images per call, and configs 4 and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07p; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-secondary > $O/prof_bench.log 2>&1 || { echo "ROCPROF FAILED"; tail $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $O/prof_bench/run_kernel_stats.csv 40 --no-load > $O/kstats_bench.txt
rm -f $O/prof_bench/run_kernel_trace.csv
head -14 $O/kstats_bench.txt
grep '^{' $O/prof_bench.log | tail -1 > $O/bench_under_rocprof.json || true
for B in 512 640; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f$B -o run -- \
    python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_f$B.log 2>&1 || { echo "PMC F $B FAILED"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w$B -o run -- \
    python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_w$B.log 2>&1 || { echo "PMC W $B FAILED"; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_f$B/run_counter_collection.csv $O/pmc_w$B/run_counter_collection.csv \
    $O/pmc_traffic_bf16x3_b$B.json 8 $B || { echo "MAP $B FAILED"; exit 1; }
done
timeout -k 10 500 python -u bench.py --beam 4 --batch 32 --tokens 256 --steps 24 --warmup 4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo "C4 FAILED"; tail $O/bench_c4.err; exit 1; }
timeout -k 10 500 python -u bench.py --arch res18trans --steps 32 --warmup 4 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED"; tail $O/bench_c5.err; exit 1; }
python -c "import json; [print(n, json.load(open('$O/bench_'+n+'.json'))['value']) for n in ('c4','c5')]"
echo done
