#!/bin/bash
# Wave-state and MFMA counters of every kernel of the update's train pass (tools/bwd_only.py), one
# rocprofv3 --pmc pass (8 SQ + 1 GRBM counters), under a hard time limit:
#   bash tools/pmc_sq.sh NAME CONFIG   -> gpurun_out/NAME/..., gpurun_out/NAME.txt (tools/pmc_sq_summary.py)
set -u
NAME=${1:-pmcsq}; CONFIG=${2:-breakout-nature-figar}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  -d $R/gpurun_out/$NAME -o run --output-format csv -- python3 $R/tools/bwd_only.py --config $CONFIG --reps 10 \
  > $R/gpurun_out/$NAME.log 2>&1
rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 $R/tools/pmc_sq_summary.py $R/gpurun_out/$NAME > $R/gpurun_out/$NAME.txt
