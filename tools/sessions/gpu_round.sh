#!/bin/bash
# One measurement pass on the GPU box (repo root), every GPU step under its own time
# limit, the first failure ends the script:
#   GPU test suite -> smoke -> headline bench (BASELINE config 2) -> rocprofv3 kernel
#   stats of a short bench -> FETCH_SIZE / WRITE_SIZE PMC passes of one encode + 8 greedy
#   steps (tools/pmc_traffic.py maps them to kernel classes).
# Usage: tools/sessions/gpu_round.sh TAG [notests]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${2:-}" != notests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 \
    || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1 \
  || { echo "ROCPROF FAILED"; tail -20 $O/prof_bench.log; exit 1; }
python3 tools/trace_phase_stats.py $O/prof_bench/run_kernel_trace.csv "mlp384_kernel<3>" 6 \
  --json $O/trace_iso_s3mlp.json > /dev/null || echo "trace phase stats failed"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- \
  python3 tools/profile_encoder.py --batch 256 --decode-steps 8 > $O/pmc_f.log 2>&1 || { echo "PMC F FAILED"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- \
  python3 tools/profile_encoder.py --batch 256 --decode-steps 8 > $O/pmc_w.log 2>&1 || { echo "PMC W FAILED"; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_f/run_counter_collection.csv $O/pmc_w/run_counter_collection.csv \
  $O/pmc_traffic_bf16x3.json 8 || echo "pmc_traffic mapping failed"
echo done
