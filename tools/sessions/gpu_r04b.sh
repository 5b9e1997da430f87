#!/bin/bash
# Round 4 profile pass: per-kernel times of one 256-row decode chain and of a 256-image
# encode (rocprofv3 --kernel-trace --stats), then the SQ counters of the encoder kernels
# (tools/gpu_pmc_kernel.sh, three passes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o run -- \
  python3 tools/decode_chain_probe.py --rows 256 --chains 1 --reps 1 > $O/dec.log 2>&1 || { echo "DEC PROF FAILED"; tail $O/dec.log; exit 1; }
python3 tools/kstats.py $O/dec/run_kernel_stats.csv 30
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/enc -o run -- \
  python3 tools/profile_encoder.py --batch 256 --encodes 2 > $O/enc.log 2>&1 || { echo "ENC PROF FAILED"; tail $O/enc.log; exit 1; }
python3 tools/kstats.py $O/enc/run_kernel_stats.csv 30
bash tools/gpu_pmc_kernel.sh r04b --batch 256
for k in "swin_attn_kernel<96" "swin_attn_kernel<192" "mlp_fused_kernel<96" "mlp_fused_kernel<192" "mlp384_kernel" "lngemm384_kernel"; do
  echo "== $k"; python3 tools/pmc_kernel.py gpurun_out/pmck_r04b "$k"
done
echo done
