#!/bin/bash
# Arbitrary PMC counters of a python tool: one rocprofv3 pass per ';'-separated group in PASSES
# (each within the per-block slot limits of MI355X_MICROARCH.md), each under its own hard limit,
# then per-kernel averages (tools/pmc_any.py) -> gpurun_out/$NAME.json.
#   NAME=x PASSES="SQ_WAVE_CYCLES SQ_BUSY_CYCLES;TCC_HIT_sum TCC_MISS_sum" bash tools/pmc_any.sh tools/bwd_only.py --config ...
set -u
NAME=${NAME:-pmc_any}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra PS <<< "${PASSES}"
i=0
for P in "${PS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $R/gpurun_out/$NAME/p$i -o run --output-format csv -- \
    python3 "$R/$1" "${@:2}" > $R/gpurun_out/$NAME.p$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($P) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i + 1))
done
python3 $R/tools/pmc_any.py $R/gpurun_out/$NAME > $R/gpurun_out/$NAME.json
