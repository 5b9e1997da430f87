#!/bin/bash
# Same-box A/B of the driver-form bench: production lib/ against one or more A/B builds
# (handwritten-math-ocr-api_amd/lib_var/NAME), interleaved, each twice.
#   TAG=s6f bash tools/sessions/gpu_ab.sh NAME [NAME...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-ab}; mkdir -p $O
L=handwritten-math-ocr-api_amd/lib_var
for rep in 1 2; do
  for v in base "$@"; do
    arg=""; [ "$v" != base ] && arg="--lib $L/$v/libmathocr.so"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $arg > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "BENCH $v FAILED"; tail $O/bench_${v}_$rep.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/bench_${v}_$rep.json')); k=d['kernel_classes']
enc=d['gpu_time_share']['encoder_ms_per_call']; dec=d['gpu_time_share']['decode_ms_per_call']
print('$v', $rep, round(d['value'],1), 'dec_step', round(d['roofline']['avg_step_ms']*1e3,1), 'enc', round(enc,2), 'dec', round(dec,2), d['config']['build'])"
  done
done
echo done
