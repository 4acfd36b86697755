#!/bin/bash
# Kernel-trace profiles of tools/bwd_only.py under several library variants (experiment builds
# written next to the product library): VARIANTS="name1 name2" -> gpurun_out/vp_<name>/.
#   VARIANTS="split bk128" CONFIG=mspacman-lstm-figar bash tools/variant_prof.sh
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS}; do
  MANETTE_HIP_LIB=$R/manette_amd/libmanette_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d $R/gpurun_out/vp_$v -o run --output-format csv -- \
    python3 $R/tools/bwd_only.py --config ${CONFIG:-mspacman-lstm-figar} --reps ${REPS:-10} > $R/gpurun_out/vp_$v.log 2>&1
  rc=$?
  echo "variant $v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
