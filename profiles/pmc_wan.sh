#!/bin/bash
# PMC passes over the WAN delta-stepping kernel (runs on the GPU box from the
# repo root): one counter group per pass, each under its own time limit.
# Usage: bash profiles/pmc_wan.sh <tag> <nsources> <variant>
set -e
R=$(pwd)
TAG=${1:-wan}
N=${2:-2048}
VAR=${3:-base}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU" \
         "SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCC_ATOMIC_sum TCC_EA0_RDREQ_sum" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -T -d $OUT/p$i -o run --output-format csv -- \
    python3 $R/profiles/quick_wan.py $N $VAR > $OUT/p$i.log 2>&1
done
cd $R
python3 profiles/pmc_summary.py $OUT ${4:-spf_dstep_kernel} > $OUT/summary.json
cat $OUT/summary.json
