#!/bin/bash
# Alternating A/B of an environment switch on bench.py lines (one box): for each config, ROUNDS x
# (A then B), each bench.py --no_cpu_baseline run under its own time limit.
#   VAR=MT_UPDATE_GATE A=0 B=1 CONFIGS="pong-nips seaquest-nature" ROUNDS=2 bash tools/ab_env_bench.sh <tag>
set -u
TAG=${1:-abenv}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in ${CONFIGS:-pong-nips}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for side in A B; do
      val=${!side}
      env $VAR=$val timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= ${BENCH_ARGS:-} \
        > $OUT/${c}_${side}_$r.log 2>&1
      rc=$?
      echo "$c $side=$val round $r rc=$rc"
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
