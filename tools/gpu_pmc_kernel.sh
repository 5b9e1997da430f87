#!/bin/bash
# SQ counters of one encode (tools/profile_encoder.py [ARGS...], e.g. --decode-steps 8),
# three passes; summarise one kernel with tools/pmc_kernel.py gpurun_out/pmck_TAG KERNEL_SUBSTRING.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
shift
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmck_$TAG/$i -o run -- python3 tools/profile_encoder.py "$@" > gpurun_out/pmck_${TAG}_$i.log 2>&1 || echo "pass $i failed" >> gpurun_out/pmck_${TAG}_fail.txt
done
exit 0
