#!/bin/bash
# Default bench (auto chain 8 x 64), the driver's 20-step form (10 x 64), GPU suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 1; }
cut -c1-330 $O/bench_default.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "BENCH DRIVER FAILED"; tail -20 $O/bench_driver.err; exit 1; }
cut -c1-330 $O/bench_driver.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
