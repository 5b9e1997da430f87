#!/bin/bash
# Round-4 final pass: GPU parity suite, smoke, the default bench and the driver's --steps 20
# form, configs 5 and 4, PMC HBM traffic at 512 / 640 images per call, rocprofv3 stats of a
# short bench, and a replicas x chain sweep of the pipeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-200 $O/bench_default.json
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "BENCH DRIVER FAILED"; tail -20 $O/bench_driver.err; exit 1; }
cut -c1-200 $O/bench_driver.json
timeout -k 10 400 python -u bench.py --arch res18trans --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err \
  || { echo "BENCH C5 FAILED"; tail -5 $O/bench_c5.err; exit 1; }
cut -c1-200 $O/bench_c5.json
timeout -k 10 500 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err \
  || { echo "BENCH C4 FAILED"; tail -5 $O/bench_c4.err; exit 1; }
cut -c1-200 $O/bench_c4.json
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
head -8 $O/kstats_bench.txt
for C in "48 2 8" "48 3 8" "40 2 10" "60 3 10" "48 2 8" "48 3 8"; do
  set -- $C
  timeout -k 10 400 python -u bench.py --steps $1 --replicas $2 --chain-batches $3 --warmup 8 --no-isolated --no-secondary --no-cpu-baseline \
    > $O/sweep_s$1r$2g$3.json 2> $O/sweep.err || { echo "SWEEP $C FAILED"; tail $O/sweep.err; exit 1; }
  echo "== steps $1 replicas $2 chain $3"; python -c "import json; d=json.load(open('$O/sweep_s$1r$2g$3.json')); print(d['value'], d['p50_call_latency_loaded_ms'])"
done
echo done
