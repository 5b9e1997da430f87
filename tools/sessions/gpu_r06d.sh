#!/bin/bash
# Round 5: SQ counters of the encoder kernels on the current tree (VERDICT r04 item 4:
# VALU per MFMA, MFMA busy, waits, LDS), one 64-image encode, three passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06d; mkdir -p $O
bash tools/gpu_pmc_kernel.sh r06d || exit 1
cat gpurun_out/pmck_r06d_fail.txt 2>/dev/null
for k in "swin_attn_kernel<96" "swin_attn_kernel<192" "mlp_fused_kernel<96" "mlp_fused_kernel<192" "mlp384_kernel" "swin_attn_noproj_kernel"; do
  echo "== $k" >> $O/pmc_encoder_kernels.txt
  python tools/pmc_kernel.py gpurun_out/pmck_r06d "$k" >> $O/pmc_encoder_kernels.txt
done
cat $O/pmc_encoder_kernels.txt | head -120
