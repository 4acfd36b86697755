#!/bin/bash
# A2 placement evidence: the same bench line under each staging mode, alternating on
# one box, with the emulator threads' staging / busy split (macro_step_host_us.emulator_threads):
#   resized   = host pool + nearest resize, 7,056*depth B per push over PCIe, the GPU stacks;
#   pooled    = host pool, the GPU resizes + stacks 84 staged rows (13,440*depth B per push);
#   zero_copy = host copies the 84 resize rows of both screens, the GPU pools + resizes + stacks
#               (26,880*depth B per push).
#   STAGINGS="resized pooled zero_copy" CONFIGS="pong-nips breakout-nature-figar" N=1 TAG=st bash tools/ab_staging.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-st}; N=${N:-1}
mkdir -p gpurun_out
for c in ${CONFIGS:-pong-nips}; do
  for i in $(seq 1 $N); do
    for st in ${STAGINGS:-resized pooled zero_copy}; do
      timeout -k 10 300 python bench.py --config $c --staging $st --no_cpu_baseline --trunk_sweep= \
        --measure_updates 0 > gpurun_out/${TAG}_${st}_${c}_$i.log 2>&1
      rc=$?
      echo "${TAG}_${st}_${c}_$i rc=$rc"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
