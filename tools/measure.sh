#!/bin/bash
# One measurement pass on the GPU box (repo root): headline bench, configs 4/5, encoder
# kernel trace, bench kernel trace and the FETCH/WRITE PMC passes for profiles/.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 python bench.py --arch res18trans --no-cpu-baseline > gpurun_out/bench_res18.json 2>> gpurun_out/bench.err
timeout -k 10 600 python bench.py --beam 4 --batch 32 --tokens 256 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_beam.json 2>> gpurun_out/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc -o run -- python3 tools/profile_encoder.py --encodes 3 > gpurun_out/prof_enc.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 tools/profile_encoder.py > gpurun_out/pmc_f.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 tools/profile_encoder.py > gpurun_out/pmc_w.log 2>&1
echo done
