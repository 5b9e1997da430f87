#!/bin/bash
# GPU test suite, then the decode chain probe.  Usage: tools/sessions/gpu_tests_probe.sh TAG [probe args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-tp}
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u tools/decode_chain_probe.py "$@" > $O/chain_probe.log 2>&1 || { echo "PROBE FAILED"; tail -20 $O/chain_probe.log; exit 1; }
cat $O/chain_probe.log
