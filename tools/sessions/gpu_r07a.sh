#!/bin/bash
# Round 5 final tree: run-to-run spread of the headline on one box (the driver's form three
# times, the default form twice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r07a; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { echo "DRIVER $i FAILED"; tail $O/bench_driver_$i.err; exit 1; }
  echo "driver $i $(python -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print(d['value'], d['p50_image_latency_ms'])")"
done
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/bench_default_$i.json 2> $O/bench_default_$i.err || { echo "DEFAULT $i FAILED"; tail $O/bench_default_$i.err; exit 1; }
  echo "default $i $(python -c "import json; d=json.load(open('$O/bench_default_$i.json')); print(d['value'], d['p50_image_latency_ms'])")"
done
echo done
