#!/bin/bash
# bench each library variant (MANETTE_HIP_LIB) on each config: VARIANTS="base wc2 ..." CONFIGS="pong-nips ..."
set -u
R=$GRAFT_REPO_ROOT
for c in ${CONFIGS:-pong-nips}; do
  for v in ${VARIANTS:-base}; do
    L=$R/manette_amd/libmanette_hip_$v.so; [ "$v" = base ] && L=$R/manette_amd/libmanette_hip.so
    MANETTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= --measure_updates 0 > gpurun_out/v_${v}_$c.log 2>&1; echo "v_${v}_$c rc=$?"
  done
done
