#!/bin/bash
# Round 6 closing measurement pass, in two calls (each under gpurun's 1200 s limit):
#   PART=a: the GPU suite, smoke, the bench in its default and driver forms, configs 4 and 5;
#   PART=b: rocprofv3 --kernel-trace --stats of the driver-form bench, FETCH_SIZE / WRITE_SIZE
#           passes of one encode + 8 greedy steps at 512 and 640 images (tools/pmc_traffic.py),
#           SQ counters of the same 640-image run (tools/gpu_pmc_kernel.sh) for s3.tail and merge1.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-s6z}; mkdir -p $O
if [ "${PART:-a}" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E 'FAILED|Error' $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "BENCH DRIVER FAILED"; tail $O/bench_driver.err; exit 1; }
  timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
  python -c "
import json
for n in ('bench_driver', 'bench'):
    d = json.load(open('$O/' + n + '.json'))
    print(n, d['value'], d['ms_per_step'], 'dec', d['roofline']['avg_step_ms'], 'p50', d['p50_image_latency_ms'],
          'serving', d.get('serving_latency_ms'), 'cpu', d['cpu_baseline']['value'], 'build', d['config']['build'])"
  timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --steps 24 --warmup 4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo "C4 FAILED"; tail $O/bench_c4.err; exit 1; }
  timeout -k 10 400 python -u bench.py --arch res18trans --steps 32 --warmup 4 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "C5 FAILED"; tail $O/bench_c5.err; exit 1; }
  python -c "import json; [print(n, json.load(open('$O/bench_'+n+'.json'))['value']) for n in ('c4','c5')]"
else
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/prof_bench.log 2>&1 || { echo "ROCPROF FAILED"; tail $O/prof_bench.log; exit 1; }
  python3 tools/kstats.py $O/prof_bench/run_kernel_stats.csv 40 --no-load > $O/kstats_bench.txt
  rm -f $O/prof_bench/run_kernel_trace.csv
  head -16 $O/kstats_bench.txt
  grep '^{' $O/prof_bench.log | tail -1 > $O/bench_under_rocprof.json || true
  for B in 512 640; do
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f$B -o run -- \
      python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_f$B.log 2>&1 || { echo "PMC F $B FAILED"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w$B -o run -- \
      python3 tools/profile_encoder.py --batch $B --decode-steps 8 > $O/pmc_w$B.log 2>&1 || { echo "PMC W $B FAILED"; exit 1; }
    python3 tools/pmc_traffic.py $O/pmc_f$B/run_counter_collection.csv $O/pmc_w$B/run_counter_collection.csv \
      $O/pmc_traffic_bf16x3_b$B.json 8 $B || { echo "MAP $B FAILED"; exit 1; }
  done
  python3 -c "
import json
d = json.load(open('$O/pmc_traffic_bf16x3_b640.json'))['classes']
for c in ('merge1', 's3.tail', 's3.attn', 'decode.step'):
    print(c, d[c]['launches'], round(d[c]['hbm_bytes_per_launch'] / 1e9, 3), 'GB per launch')"
  bash tools/gpu_pmc_kernel.sh ${TAG:-s6z} --batch 640
  [ -s gpurun_out/pmck_${TAG:-s6z}_fail.txt ] && { echo "SQ PASS FAILED"; cat gpurun_out/pmck_${TAG:-s6z}_fail.txt; exit 1; }
  for k in "mlp384_kernel<3, true" "merge1_kernel" "swin_attn_noproj_kernel"; do
    echo "== $k"; python3 tools/pmc_kernel.py gpurun_out/pmck_${TAG:-s6z} "$k"
  done > $O/sq_counters.txt
  cat $O/sq_counters.txt
fi
echo done
