#!/bin/bash
# GPU gate: the -m gpu suite, the driver's smoke, one default bench line.  Every GPU step
# has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
if [ "${2:-bench}" = bench ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  cut -c1-600 gpurun_out/${TAG}_bench.json
fi
