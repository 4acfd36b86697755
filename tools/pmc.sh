#!/bin/bash
# HBM traffic of every kernel of a short bench run, from rocprofv3 PMC counters: one pass per
# counter (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass), each under its
# own hard time limit. Output: gpurun_out/$NAME/{fetch,write}/.../counter_collection.csv and
# gpurun_out/$NAME.json (tools/pmc_summary.py: per-kernel averages, gfx950 FETCH_SIZE x2).
set -u
NAME=${1:-pmc}
shift || true
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d $R/gpurun_out/$NAME/$C -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no_cpu_baseline --trunk_sweep= "$@" > $R/gpurun_out/$NAME.$C.log 2>&1
  rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/$NAME > $R/gpurun_out/$NAME.json
