#!/bin/bash
# Round 5, first box: the whole -m gpu suite on the current tree (late logit windows,
# chain-length bitwise test, int16 scale masking), then the default bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -h "PARITY_RECORD" $O/tests.log | cut -c1-260
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d.get('roofline'))"
echo done
