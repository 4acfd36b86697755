#!/bin/bash
# A/B of library variants on one box (MANETTE_HIP_LIB), alternating N times per config:
#   VARIANTS="base cp" CONFIGS="breakout-nature-figar" N=3 TAG=abcp bash tools/ab_lib.sh
# base = the product libmanette_hip.so; v = manette_amd/libmanette_hip_<v>.so. Logs:
# gpurun_out/<TAG>_<v>_<config>_<i>.log. A fault-like exit stops the loop.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-ablib}; N=${N:-3}
mkdir -p gpurun_out
for c in ${CONFIGS:-pong-nips}; do
  for i in $(seq 1 $N); do
    for v in ${VARIANTS:-base}; do
      L=$R/manette_amd/libmanette_hip_$v.so; [ "$v" = base ] && L=$R/manette_amd/libmanette_hip.so
      MANETTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= \
        --measure_updates 0 > gpurun_out/${TAG}_${v}_${c}_$i.log 2>&1
      rc=$?
      echo "${TAG}_${v}_${c}_$i rc=$rc"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
