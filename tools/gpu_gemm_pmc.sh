#!/bin/bash
# SQ/TA counters for one GEMM shape under two kernel variants (tools/gemm_bench)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPE="9216 3072 768 3 1 5"
i=0
for v in "MOCR_GEMM_STAG_MIN=1" "MOCR_GEMM_BIG_MIN=0"; do
  for set in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
             "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum"; do
    i=$((i+1))
    env $v timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/gp/$i -o a -- ./tools/gemm_bench $SHAPE > gpurun_out/gp_$i.log 2>&1
    echo "$i $v $set" >> gpurun_out/gp_index.txt
  done
done
exit 0
