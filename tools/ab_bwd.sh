#!/bin/bash
# A/B of the update's train pass between library variants: rocprofv3 kernel traces of
# tools/bwd_only.py (REPS back-to-back train_backward calls of the benchmarked learner) per variant
# and config, then the per-kernel summary of each (tools/prof_summary.py).
#   VARIANTS="stream gen" CONFIGS="seaquest-nature breakout-nature-figar" bash tools/ab_bwd.sh <tag>
# variant v = manette_amd/libmanette_hip_<v>.so (base = the product library)
set -u
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in ${CONFIGS:-seaquest-nature}; do
  for v in ${VARIANTS:-base}; do
    L=$R/manette_amd/libmanette_hip_$v.so; [ "$v" = base ] && L=$R/manette_amd/libmanette_hip.so
    D=$R/gpurun_out/${TAG}_${v}_$c
    (cd /tmp && MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
      python3 $R/tools/bwd_only.py --config $c --reps ${REPS:-20} > $D.log 2>&1)
    rc=$?
    echo "${TAG}_${v}_$c rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    f=$(find $D -name '*kernel_trace.csv' | head -1)
    [ -n "$f" ] && python3 $R/tools/prof_summary.py $f > $D.summary.txt
  done
done
exit 0
