#!/bin/bash
# Config 4 (beam) and config 5 (ResNet18-trans) after moving the engine-setup memsets off
# the null stream, a kernel trace of the beam bench (hardware queues per replica), the
# beam / res18 GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --no-secondary --steps 24 > $O/beam.json 2> $O/beam.err \
  || { echo "BEAM FAILED"; tail $O/beam.err; exit 1; }
cut -c1-200 $O/beam.json
timeout -k 10 400 python -u bench.py --arch res18trans --no-cpu-baseline --no-secondary --steps 64 > $O/res18.json 2> $O/res18.err \
  || { echo "RES18 FAILED"; tail $O/res18.err; exit 1; }
cut -c1-200 $O/res18.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cur -o run -- python3 bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --no-secondary --steps 8 --warmup 4 --no-isolated > $O/cur.log 2>&1 || { echo trace failed; exit 1; }
python3 tools/trace_busy.py $O/cur/run_kernel_trace.csv beam_select
timeout -k 10 400 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_res18.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
