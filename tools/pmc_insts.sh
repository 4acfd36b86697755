#!/bin/bash
# Instruction-class counters of the update's train pass (tools/bwd_only.py): where a kernel's issue
# slots go (VALU / MFMA / LDS / SALU / VMEM instructions, LDS stalls and bank conflicts). Lists the
# device's counters first (gpurun_out/$NAME.counters.txt) and keeps only candidates it has, at most
# 8 SQ counters per pass (MI355X_MICROARCH.md PMC slots), each pass under its own hard limit.
#   bash tools/pmc_insts.sh NAME CONFIG   -> gpurun_out/NAME.json (tools/pmc_any.py)
set -u
NAME=${1:-pmcinsts}; CONFIG=${2:-mspacman-lstm-figar}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/$NAME.counters.txt 2>&1
echo "list rc=$?"
pick() {  # the candidates the device lists, space-separated
  local out=""
  for c in "$@"; do
    grep -q -w "$c" $R/gpurun_out/$NAME.counters.txt && out="$out $c"
  done
  echo $out
}
P0=$(pick SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES)
P1=$(pick SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY)
echo "pass0: $P0"
echo "pass1: $P1"
i=0
for P in "$P0" "$P1"; do
  [ -z "$P" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $P -d $R/gpurun_out/$NAME/p$i -o run --output-format csv -- \
    python3 $R/tools/bwd_only.py --config $CONFIG --reps 10 > $R/gpurun_out/$NAME.p$i.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i + 1))
done
python3 $R/tools/pmc_any.py $R/gpurun_out/$NAME > $R/gpurun_out/$NAME.json
rc=$?
rm -rf $R/gpurun_out/$NAME
exit $rc
