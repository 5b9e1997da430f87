#!/bin/bash
# rocprofv3 kernel stats of the beam bench: round-2 tree (tmp_r02) vs current
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bp
(cd tmp_r02 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/bp/r02 -o run -- python3 bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 4 --warmup 1 --no-isolated > ../gpurun_out/bp/r02.log 2>&1) || { echo r02 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp/cur -o run -- python3 bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 4 --warmup 1 --no-isolated > gpurun_out/bp/cur.log 2>&1 || { echo cur failed; exit 1; }
rm -f gpurun_out/bp/*/run_kernel_trace.csv
echo "== r02"; python3 tools/kstats.py gpurun_out/bp/r02/run_kernel_stats.csv 14
echo "== cur"; python3 tools/kstats.py gpurun_out/bp/cur/run_kernel_stats.csv 14
