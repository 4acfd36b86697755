#!/bin/bash
# One round's measurement set on the GPU box (profiles/<tag>): every config's bench line with its
# CPU baseline (tools/bench_all.sh), the rocprof kernel summary of each bench command
# (tools/prof_all.sh), and the PMC HBM traffic of the NATURE roofline launch (tools/pmc_trunk.sh;
# Pong's is profiles/pmc_trunk_pong-nips.json). Each step under its own time limit; stops on failure.
#   bash tools/measure_round.sh r04k
set -u
TAG=${1:-meas}
CPU_ALL=1 TAG=$TAG bash tools/bench_all.sh || exit $?
bash tools/prof_all.sh $TAG || exit $?
for c in ${PMC_CONFIGS:-breakout-nature-figar seaquest-nature breakout-pwyx-figar-rgb}; do
  bash tools/pmc_trunk.sh pmc_trunk_$c --config $c || exit $?
done
