#!/bin/bash
# A/B of the bench on one box under two settings of an env var: VAR=A vs VAR=B, alternating N times
set -u
VAR=${VAR:-MH_WARM_NEXT}; A=${A:-0}; B=${B:-1}; ARGS=${ARGS:-}; TAG=${TAG:-ab}; N=${N:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --no_cpu_baseline --trunk_sweep= --measure_updates 0 $ARGS > gpurun_out/${TAG}_${v}_$i.log 2>&1; echo "$VAR=$v $i rc=$?"
  done
done
