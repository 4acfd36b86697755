#!/bin/bash
# PMC traffic of every config's roofline launch at the round's last code (bench.py reads
# profiles/pmc_trunk_<config>.json as roofline.traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in pong-nips seaquest-nature breakout-nature-figar breakout-pwyx-figar-rgb mspacman-lstm-figar; do
  bash tools/pmc_trunk.sh pmc_trunk_$c --config $c --reps 50 > gpurun_out/r06pm_$c.log 2>&1 || exit 1
done
