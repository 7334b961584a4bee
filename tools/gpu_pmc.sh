#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c3 metric}; do
 i=0
 for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
   i=$((i+1))
   timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $O/pmc_${c}_$i -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/pmc_${c}_$i.log 2>&1 || { echo "pmc $c $i failed"; tail -5 $O/pmc_${c}_$i.log; exit 1; }
 done
 echo "== $c"; python3 $R/tools/pmc_summary.py $O/pmc_${c}_1 $O/pmc_${c}_2 $O/pmc_${c}_3
done
