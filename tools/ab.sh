#!/bin/bash
# A/B of the bench on one box: the scratch/r01 worktree (round-1 code) vs this tree
set -u
mkdir -p gpurun_out
for i in 1 2; do
  (cd scratch/r01 && timeout -k 10 200 python bench.py --no_cpu_baseline --trunk_sweep= > ../../gpurun_out/ab_old_$i.log 2>&1); echo "old $i rc=$?"
  timeout -k 10 200 python bench.py --no_cpu_baseline --trunk_sweep= --measure_updates 0 > gpurun_out/ab_new_$i.log 2>&1; echo "new $i rc=$?"
done
