#!/bin/bash
# A/B of host-runner library variants on one box, alternating: VARIANTS names libmanette_host_<v>.so
# (base = the product library), copied over libmanette_host.so for each run (the HIP library loads it
# by name from its own directory) and restored at the end. ENV_<v> (e.g. ENV_pd4="MH_PREFETCH_ROWS=4")
# adds environment settings to a variant's runs.
#   VARIANTS="old base" CONFIGS="pong-nips" N=2 TAG=abh bash tools/ab_host.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-abh}; N=${N:-2}
mkdir -p gpurun_out
cp $R/manette_amd/libmanette_host.so /tmp/libmanette_host_base.so
rc_all=0
for c in ${CONFIGS:-pong-nips}; do
  for i in $(seq 1 $N); do
    for v in ${VARIANTS:-old base}; do
      src=$R/manette_amd/libmanette_host_$v.so; [ "$v" = base ] && src=/tmp/libmanette_host_base.so
      [ -f "$src" ] || src=/tmp/libmanette_host_base.so
      cp $src $R/manette_amd/libmanette_host.so
      ev=ENV_$v; extra=${!ev:-}
      env $extra timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= --measure_updates 0 \
        ${BENCH_ARGS:-} > gpurun_out/${TAG}_${v}_${c}_$i.log 2>&1
      rc=$?
      echo "${TAG}_${v}_${c}_$i rc=$rc"
      if [ $rc -ne 0 ]; then rc_all=$rc; break 3; fi
    done
  done
done
cp /tmp/libmanette_host_base.so $R/manette_amd/libmanette_host.so
exit $rc_all
