#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run with a variant library (tools only):
#   bash tools/prof_lib.sh NAME LIB [bench args]   (LIB: path of a libmanette_hip variant)
set -u
NAME=$1; LIB=$2; shift 2
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp MANETTE_HIP_LIB=$LIB
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$NAME -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 10 --no_cpu_baseline --trunk_sweep= "$@" > $R/gpurun_out/$NAME.log 2>&1
rc=$?
echo "rocprof rc=$rc"
f=$(ls $R/gpurun_out/$NAME/*/run_kernel_trace.csv $R/gpurun_out/$NAME/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $R/tools/prof_summary.py $f > $R/gpurun_out/$NAME.summary.txt
exit $rc
