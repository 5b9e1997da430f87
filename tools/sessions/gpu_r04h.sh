#!/bin/bash
# FFN fold GEMM prefetch ring (two k steps in flight above 256 workgroups): decode chain
# A/B against lib_var/base (HEAD) at 256-640 rows, and kernel stats at 640 rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04h; mkdir -p $O
for L in new base; do
  A=""; [ $L = base ] && A="--lib handwritten-math-ocr-api_amd/lib_var/base/libmathocr.so"
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 256,512,640 --chains 1 --reps 2 $A > $O/rows_$L.log 2>&1 \
    || { echo "ROWS $L FAILED"; tail $O/rows_$L.log; exit 1; }
  timeout -k 10 300 python -u tools/decode_chain_probe.py --rows 512,640 --chains 2 --reps 2 $A > $O/rows2_$L.log 2>&1 \
    || { echo "ROWS2 $L FAILED"; tail $O/rows2_$L.log; exit 1; }
  echo "== $L"; grep -h rows_per_s $O/rows_$L.log $O/rows2_$L.log | cut -c1-140
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec640 -o run -- \
  python3 tools/decode_chain_probe.py --rows 640 --chains 1 --reps 1 > $O/dec640.log 2>&1 || { echo "PROF FAILED"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "b256_chain or wide_chain or teacher_forced or config2" > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in production s2o3; do
  A=""; [ $L = s2o3 ] && A="--lib handwritten-math-ocr-api_amd/lib_var/s2o3/libmathocr.so"
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.,s2. $A > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== ops $L"; tail -12 $O/ops_$L.log
done
echo done
