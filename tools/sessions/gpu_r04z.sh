#!/bin/bash
# Round-4 pass on the current tree: GPU parity suite, smoke, the default bench (64 steps,
# with the isolated / literal-config-2 / CPU-baseline passes) and the driver's --steps 20
# form; PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of one encode + 8 greedy steps at
# 512 and 640 images per call; rocprofv3 --kernel-trace --stats of a short bench; and the
# stage-1/2 attention with its weight loads removed (wp5 timing probe, wrong results).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "BENCH DRIVER FAILED"; tail -20 $O/bench_driver.err; exit 1; }
cut -c1-300 $O/bench_driver.json
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
for L in production wp5; do
  A=""; [ $L != production ] && A="--lib handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so"
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production $A > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|total" $O/ops_$L.log
done
echo done
