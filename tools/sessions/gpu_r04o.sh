#!/bin/bash
# Where the fused stage-1/2 attention kernels spend their time: per-op times of a 512-image
# encode with each timing probe of swin_attn_kernel (-DMOCR_WATTN_PROBE=N, wrong results).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04o; mkdir -p $O
for L in production wp1 wp2 wp3 wp4 wp5; do
  A=""; [ $L != production ] && A="--lib handwritten-math-ocr-api_amd/lib_var/$L/libmathocr.so"
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 3 --variants production --filter s1.attn,s2.attn $A > $O/ops_$L.log 2>&1 \
    || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn" $O/ops_$L.log
done

timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_full.py -k "640_chain" > $O/test640.log 2>&1 \
  || { echo "TEST640 FAILED"; tail -30 $O/test640.log; exit 1; }
tail -3 $O/test640.log
echo done
