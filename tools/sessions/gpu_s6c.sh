#!/bin/bash
# Round 6: the whole GPU suite on the tree with the stage-3 block tail kernel (mlp384 PROJ),
# the micro-batched /predict and the uneven-shard gather; smoke; the bench in both forms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-s6c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E 'FAILED|Error|error' $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "BENCH DRIVER FAILED"; tail $O/bench_driver.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_driver.json')); k=d['kernel_classes']
print('driver', d['value'], d['ms_per_step'], 'dec', d['roofline']['avg_step_ms'], 'gemm', d['roofline_gemm']['kernel'], d['roofline_gemm']['frac'])
print({c: round(v['avg_ms']*v['launches']/3, 3) for c, v in k.items() if c.startswith('s3')})
print('p50', d['p50_image_latency_ms'], d['image_latency_samples'], 'serving', d.get('serving_latency_ms'), 'build', d['config']['build'])"
echo done
