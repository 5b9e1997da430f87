#!/bin/bash
# Round 5: mlp.hip / wattn.hip built with -fno-slp-vectorize (no packed f32 VALU beside the
# MFMAs) vs production: per-op times of a 512-image encode, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06o; mkdir -p $O
lib() { [ $1 = production ] && echo "" || echo "--lib handwritten-math-ocr-api_amd/lib_var/$1/libmathocr.so"; }
for L in production noslp_mlp noslp_wattn production noslp_mlp noslp_wattn; do
  timeout -k 10 300 python -u tools/op_times.py --batch 512 --encodes 2 --variants production --filter s1.,s2.,s3. $(lib $L) \
    > $O/ops_$L.log 2>&1 || { echo "OPS $L FAILED"; tail $O/ops_$L.log; exit 1; }
  echo "== $L"; grep -E "attn|mlp|total" $O/ops_$L.log
done
echo done
