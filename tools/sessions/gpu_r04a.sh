#!/bin/bash
# Round 4 first pass: the new conditioning / NaN tests, the GPU suite, the driver's bench
# form with the auto chain (5 x 64) and with 4 x 64, and the no-launcher 2-rank bench.
set -o pipefail
mkdir -p gpurun_out/r04a
O=gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_gpu_conditioning.py -x -v -rP --timeout 120 --timeout-method thread \
  > $O/cond.log 2>&1 || { echo "COND FAILED"; tail -40 $O/cond.log; exit 1; }
grep -E "PARITY_RECORD|passed|failed" $O/cond.log | tail -12
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in production cn; do
  A=""; [ $L = cn ] && A="--lib handwritten-math-ocr-api_amd/lib_var/cn/libmathocr.so"
  timeout -k 10 240 python -u tools/decode_chain_probe.py --rows 256 --chains 1,2 --reps 2 $A > $O/chain_$L.log 2>&1 \
    || { echo "CHAIN $L FAILED"; tail -20 $O/chain_$L.log; exit 1; }
  echo "$L"; grep rows_per_s $O/chain_$L.log
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_auto.json 2> $O/bench_auto.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_auto.err; exit 1; }
cut -c1-300 $O/bench_auto.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --chain-batches 4 --no-cpu-baseline --no-secondary \
  > $O/bench_g4.json 2> $O/bench_g4.err || { echo "BENCH G4 FAILED"; tail -20 $O/bench_g4.err; exit 1; }
cut -c1-300 $O/bench_g4.json
timeout -k 10 400 python -u bench.py --gpus 2 --steps 8 --warmup 4 --no-cpu-baseline \
  > $O/bench_n2.json 2> $O/bench_n2.err || { echo "BENCH N2 FAILED"; tail -20 $O/bench_n2.err; exit 1; }
cut -c1-400 $O/bench_n2.json
echo done
