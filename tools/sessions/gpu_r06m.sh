#!/bin/bash
# Round 5: timing probes of the fused attention kernels (wrong results, times only):
# MOCR_WATTN_PROBE 1 no X loads, 2 no qkv MFMAs, 5 no weight loads; per-op times of a
# 512-image encode against production.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06m; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production wp1 wp2 wp5 production; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 2 --variants production --filter s1.,s2.,s3. $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|proj|total" $O/ops_$L.log
done
echo done
