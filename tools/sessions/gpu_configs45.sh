#!/bin/bash
# BASELINE configs 5 (ResNet18-trans, B = 64) and 4 (beam 4, B = 32, 256 tokens) on the
# current tree.  Usage: tools/sessions/gpu_configs45.sh TAG
set -o pipefail
mkdir -p gpurun_out
T=${1:-c45}
timeout -k 10 400 python -u bench.py --arch res18trans --no-cpu-baseline > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err || { tail -5 gpurun_out/${T}_bench_c5.err; exit 1; }
cut -c1-200 gpurun_out/${T}_bench_c5.json
timeout -k 10 500 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { tail -5 gpurun_out/${T}_bench_c4.err; exit 1; }
cut -c1-200 gpurun_out/${T}_bench_c4.json
