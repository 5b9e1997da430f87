#!/bin/bash
# Round 5: counters of the encoder kernels on the current tree (VALU
# per MFMA, MFMA busy, waits, LDS; and the memory path: TA / TD busy, L1 and L2 hits), one
# 64-image encode, one pass per counter set.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06d; mkdir -p $O
bash tools/gpu_pmc_kernel.sh r06d || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmck_r06d/4 -o run -- python3 tools/profile_encoder.py > gpurun_out/pmck_r06d_4.log 2>&1 || echo "pass 4 failed" >> gpurun_out/pmck_r06d_fail.txt
cat gpurun_out/pmck_r06d_fail.txt 2>/dev/null
for k in "swin_attn_kernel<96" "swin_attn_kernel<192" "mlp_fused_kernel<96" "mlp_fused_kernel<192" "mlp384_kernel" "swin_attn_noproj_kernel" "gemm_x3_stagq"; do
  echo "== $k" >> $O/pmc_encoder_kernels.txt
  python tools/pmc_kernel.py gpurun_out/pmck_r06d "$k" >> $O/pmc_encoder_kernels.txt
done
cat $O/pmc_encoder_kernels.txt | head -150
