#!/bin/bash
# GPU test suite + smoke + default bench, each under its own time limit; the first
# failure ends the script.  Usage: tools/sessions/gpu_quick.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
echo done
