#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run; output under gpurun_out/$1
set -u
NAME=${1:-prof}
shift || true
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$NAME -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 10 --no_cpu_baseline --trunk_sweep= "$@" > $R/gpurun_out/$NAME.log 2>&1
echo "rocprof rc=$?"
